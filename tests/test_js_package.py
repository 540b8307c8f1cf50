"""The JS drop-in package (fluidframework_amd/js: index.js over the N-API addon mtb_napi.node).

CPU: the addon loads, exposes one function per C-ABI entry point, packs all 30 reference replay logs
through Client.applyMsg, keeps the reference's assert text (0x038) and fails loudly without a GPU.
GPU: node replays the 30 reference logs (client.replay.spec.ts style) and checks the text after every
group, through both flush() and the thread-pool flushAsync(); then Client.load(runtime, storage) of
every document's summary (and of a committed reference summary) summarizes back to the same bytes.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "fluidframework_amd", "js")
ADDON = os.path.join(JS, "mtb_napi.node")

needs_node = pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(ADDON),
                                reason="node or the built addon is not available")


def _node(*args, timeout=240):
    r = subprocess.run(["node", os.path.join(JS, "test", "parity.js"), *args], capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@needs_node
def test_js_package_cpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (the CPU check expects MTB_E_NODEV)")
    out = _node("--cpu")
    assert "js cpu checks ok: 30 logs packed" in out
    assert "js cpu checks ok: summary load packed" in out


@needs_node
@pytest.mark.gpu
def test_js_package_replays_reference_logs_on_gpu(tmp_path):
    import json
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import OracleMatrix
    o = OracleMatrix()
    o.start_collab("obs")
    for m in json.load(open(os.path.join(JS, "test", "matrix_log.json"))):
        o.apply_msg(m)
    exp = o.summarize()
    nr, nc = o.rows.get_length(), o.cols.get_length()
    exp["cells"] = [[r, c, o.get_cell(r, c)] for r in range(nr) for c in range(nc)]
    path = tmp_path / "matrix_expect.json"
    path.write_text(json.dumps(exp))
    # SnapshotLegacy + tracked catch-up messages of the 30 reference logs (oracle, sequence.ts:697-748)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import msg_from_compact, replay_fixtures
    from pyoracle import OracleDoc
    legacy = []
    for _, d in replay_fixtures():
        o = OracleDoc()
        o.insert_text_local(0, d["initialText"])
        o.start_collab("A")
        o.enable_catch_up()
        for g in d["groups"]:
            for m in g["msgs"]:
                o.apply_msg(msg_from_compact(m))
        legacy.append(o.summarize_legacy())
    lpath = tmp_path / "legacy_expect.json"
    lpath.write_text(json.dumps(legacy))
    os.environ["MTB_JS_MATRIX_EXPECT"] = str(path)
    os.environ["MTB_JS_LEGACY_EXPECT"] = str(lpath)
    try:
        out = _node()
    finally:
        del os.environ["MTB_JS_MATRIX_EXPECT"]
        del os.environ["MTB_JS_LEGACY_EXPECT"]
    assert "js gpu legacy ok" in out
    assert "js gpu parity ok" in out
    assert "js gpu load ok" in out
    assert "js gpu matrix ok" in out


@needs_node
@pytest.mark.gpu
def test_js_live_clients_on_gpu(tmp_path):
    """Live clients through the JS package (insert / remove / annotate local ops, their acks and reconnects
    through regeneratePendingOp): every client's text
    after every round equals its oracle client's (tests/helpers.run_local_farm)."""
    import json
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import run_local_farm
    rec = {}
    run_local_farm(7, n_clients=3, n_rounds=30, annotate=True, record=rec, new_mode=True, reconnect=0.3)
    path = tmp_path / "farm.json"
    assert any(kind == "regen" for rnd in rec["rounds"] for ev, _, _ in rnd for kind, _ in ev)
    path.write_text(json.dumps({"ids": rec["ids"], "initial": "hello world", "newMode": True,
                                "rounds": [[ev for ev, _, _ in rnd] for rnd in rec["rounds"]]}))
    r = subprocess.run(["node", os.path.join(JS, "test", "local_farm.js"), str(path)], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    want = [[t for _, _, t in rnd] for rnd in rec["rounds"]]
    assert got["texts"] == want
    assert [int(h, 16) for h in got["digests"]] == [d for _, d, _ in rec["rounds"][-1]]


@needs_node
@pytest.mark.gpu
def test_js_client_api_on_gpu():
    """TestClient helpers, getText ranges, Client.annotateMarker (pending keys, ack) and a remote relative op
    through the JS package: text, the op it returns and the state digest equal the oracle's."""
    import json
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyoracle import OracleDoc
    r = subprocess.run(["node", os.path.join(JS, "test", "client_api.js")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got["ranges"] == ["abhello world", "ab", "he", "ello world"]
    want_op = {"props": {"color": "red"}, "relativePos1": {"id": "m", "before": True}, "relativePos2": {"id": "m"}, "type": 2}
    assert got["op"] == want_op
    o = OracleDoc(new_length_calc=True)
    o.insert_text_local(0, "hello world")
    o.start_collab("me")
    mk = lambda op, seq, ref, cid: {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,  # noqa: E731
                                    "minimumSequenceNumber": 0, "type": "op", "contents": op}
    o.apply_msg(mk({"pos1": 0, "seg": "ab", "type": 0}, 1, 0, "a"))
    o.apply_msg(mk({"pos1": 2, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m"}}, "type": 0}, 2, 1, "b"))
    assert o.local_op_json(want_op) == want_op
    o.apply_msg(mk({"pos1": 0, "pos2": 4, "props": {"color": "blue", "w": 1}, "type": 2}, 3, 2, "a"))
    o.apply_msg(mk(want_op, 4, 2, "me"))
    o.apply_msg(mk({"relativePos1": {"id": "m"}, "seg": "!", "type": 0}, 5, 4, "b"))
    assert got["text"] == o.get_text()
    assert int(got["digest"], 16) == o.digest()
