"""GPU parity of SnapshotV1 load (Client.load -> SnapshotLoader, snapshotLoader.ts:41-257).

The engine reloads the header on the host into the device tree layout and appends the body chunks on
the GPU (LOADSEG records through the insert walk).  Bar: bit-exact against the CPU oracle's restatement
of the loader — canonical segment dumps (tree shape included), text, and the SnapshotV1 summary written
back — on:
* the 6 committed reference summaries (which must also round-trip to their own bytes);
* the 30 reference replay logs summarized mid-stream and loaded, then the rest of each log replayed
  (text checked against the reference's golden text);
* synthetic multi-client logs summarized mid-stream, both length-calculation modes;
* constructed summaries with removals above the MSN (NonCollab segments removed by several clients) in
  header and body chunks, and client segments above the MSN in the header, followed by remote ops;
* the reference's own failure: a body append that lands outside the (refSeq 0, client) view throws
  "MergeTree insert failed" on both sides.
"""
import random

import pytest

from helpers import (first_diff, make_v1_summary, msg_from_compact, records_to_msgs, replay_fixtures,
                     snapshot_fixture)

pytestmark = pytest.mark.gpu

FIXTURES = ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations", "withIntervals"]


def _batch(n, **kw):
    from fluidframework_amd import MergeTreeBatch
    return MergeTreeBatch(n, **kw)


def _same(B, i, o, what):
    gd, od = B.dump_segments(i), o.dump_segments()
    assert gd == od, f"{what}: segment dump differs: {first_diff(gd, od)}"
    assert B.text(i) == o.get_text(), f"{what}: text differs"
    gb, gs = B.summarize_v1(i)
    osum = o.summarize_v1()
    assert [list(x) for x in gb] == osum["blobs"], f"{what}: SnapshotV1 blobs differ"
    assert gs == osum["summary"], f"{what}: ISummaryTreeWithStats differs"


def test_reference_summaries_load_and_round_trip():
    from pyoracle import OracleDoc
    B = _batch(len(FIXTURES))
    for i, name in enumerate(FIXTURES):
        B[i].load(snapshot_fixture(name))
    B.flush()
    for i, name in enumerate(FIXTURES):
        o = OracleDoc()
        o.load_v1(snapshot_fixture(name), "snapshot")
        gd, od = B.dump_segments(i), o.dump_segments()
        assert gd == od, f"{name}: segment dump differs: {first_diff(gd, od)}"
        assert B.text(i) == o.get_text()
        blobs, _ = B.summarize_v1(i, 0, 0)
        assert [list(x) for x in blobs] == snapshot_fixture(name), f"{name}: summary does not round-trip"


@pytest.mark.parametrize("cut", [16, 40])
def test_reference_logs_load_mid_stream_then_continue(cut):
    from pyoracle import OracleDoc
    fx = replay_fixtures()
    B = _batch(len(fx))
    oracles = []
    for i, (_, d) in enumerate(fx):
        a = OracleDoc()
        a.insert_text_local(0, d["initialText"])
        a.start_collab("A")
        for g in d["groups"][:cut]:
            for m in g["msgs"]:
                a.apply_msg(msg_from_compact(m))
        blobs = [list(x) for x in a.summarize_v1()["blobs"]]
        B[i].load(blobs, "A")
        o = OracleDoc()
        o.load_v1(blobs, "A")
        oracles.append(o)
    B.flush()
    for i, (name, d) in enumerate(fx):
        assert B[i].getText() == d["groups"][cut - 1]["resultText"], f"{name}: text right after load"
        _same(B, i, oracles[i], f"{name} loaded at group {cut}")
    for i, (_, d) in enumerate(fx):
        for g in d["groups"][cut:]:
            for m in g["msgs"]:
                B[i].applyMsg(msg_from_compact(m))
                oracles[i].apply_msg(msg_from_compact(m))
    B.flush()
    for i, (name, d) in enumerate(fx):
        assert B[i].getText() == d["groups"][-1]["resultText"], f"{name}: final text"
        _same(B, i, oracles[i], f"{name} loaded at group {cut}, replayed to the end")


@pytest.mark.parametrize("new_mode", [False, True])
def test_synthetic_logs_load_mid_stream_then_continue(new_mode):
    from pyoracle import OracleDoc
    from pyloggen import LogBatch, make_cfg
    cfg = make_cfg(seed=31 + int(new_mode), n_ops=1500, new_length_calc=new_mode)
    lb = LogBatch(cfg, 0, 24)
    props = lb.props_json()
    B = _batch(lb.n, new_length_calc=new_mode)
    oracles, rests = [], []
    for i in range(lb.n):
        tb = lb.doc_text_bytes(i)
        il = lb.docs[i].initial_len
        msgs = records_to_msgs(lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb, props, lb.client_ids(i))
        cut = len(msgs) // 3 + 37 * i
        a = OracleDoc(new_length_calc=new_mode)
        a.insert_text_local(0, tb[: il * 2].decode("utf-16-le"))
        a.start_collab("obs")
        for m in msgs[:cut]:
            a.apply_msg(m)
        blobs = [list(x) for x in a.summarize_v1()["blobs"]]
        B[i].load(blobs, "obs")
        o = OracleDoc(new_length_calc=new_mode)
        o.load_v1(blobs, "obs")
        oracles.append(o)
        rests.append(msgs[cut:])
    B.flush()
    for i in range(lb.n):
        _same(B, i, oracles[i], f"doc {i} after load")
        for m in rests[i]:
            B[i].applyMsg(m)
            oracles[i].apply_msg(m)
    B.flush()
    for i in range(lb.n):
        _same(B, i, oracles[i], f"doc {i} after load + tail")


def _remote_tail(o, seed, n_ops, start_seq, msn, clients):
    """Valid remote ops after a load: each author has seen everything (refSeq = current seq)."""
    rng = random.Random(seed)
    msgs = []
    seq = start_seq
    for _ in range(n_ops):
        seq += 1
        ln = o.get_length()
        r = rng.random()
        if ln == 0 or r < 0.5:
            contents = {"type": 0, "pos1": rng.randint(0, ln), "seg": "".join(rng.choice("xyz\n") for _ in range(rng.randint(1, 6)))}
        else:
            p1 = rng.randint(0, ln - 1)
            p2 = min(ln, p1 + rng.randint(1, 8))
            contents = {"type": 1, "pos1": p1, "pos2": p2} if r < 0.8 else \
                {"type": 2, "pos1": p1, "pos2": p2, "props": {"bold": rng.choice([True, None])}}
        m = {"clientId": rng.choice(clients), "sequenceNumber": seq, "referenceSequenceNumber": seq - 1,
             "minimumSequenceNumber": msn, "type": "op", "contents": contents}
        o.apply_msg(m)
        msgs.append(m)
    return msgs


@pytest.mark.parametrize("new_mode", [False, True])
def test_constructed_summaries_with_removals_in_header_and_body(new_mode):
    from pyoracle import OracleDoc
    n = 16
    B = _batch(n, new_length_calc=new_mode)
    oracles, tails, sums = [], [], []
    for i in range(n):
        sums.append(make_v1_summary(100 + i, 300 + 40 * i, 250, 10, 40, p_removed=0.3))
    B.load_v1_many(list(range(n)), sums, ["obs"] * n, threads=4)  # the parallel host path
    for i in range(n):
        blobs = sums[i]
        o = OracleDoc(new_length_calc=new_mode)
        o.load_v1(blobs, "obs")
        oracles.append(o)
    B.flush()
    for i in range(n):
        _same(B, i, oracles[i], f"constructed summary {i}")
        tails.append(_remote_tail(oracles[i], 7 * i, 200, 40, 10, ["client-0", "client-1", "client-5"]))
        for m in tails[i]:
            B[i].applyMsg(m)
    B.flush()
    for i in range(n):
        _same(B, i, oracles[i], f"constructed summary {i} + 200 remote ops")


def test_load_failure_matches_reference():
    """Client segments above the MSN in the header shrink the (refSeq 0, client) view the body is appended
    in: for some summaries the reference throws "MergeTree insert failed"; the engine must agree doc by doc."""
    from fluidframework_amd import MergeTreeError
    from pyoracle import OracleDoc
    outcomes = []
    for seed in range(20):
        blobs = make_v1_summary(seed, 400, 300, 10, 40, p_client=0.2)
        o = OracleDoc()
        try:
            o.load_v1(blobs, "obs")
            o.get_text()
            ok = True
        except Exception as e:
            assert "MergeTree insert failed" in str(e)
            ok = False
        B = _batch(1)
        B[0].load(blobs, "obs")
        if ok:
            B.flush()
            _same(B, 0, o, f"seed {seed}")
        else:
            with pytest.raises(MergeTreeError, match="MergeTree insert failed"):
                B.flush()
        outcomes.append(ok)
    assert any(outcomes) and not all(outcomes)


def test_rewind_restores_loaded_documents():
    from pyoracle import OracleDoc
    blobs = make_v1_summary(5, 500, 200, 10, 40, p_removed=0.3)
    B = _batch(2)
    B[0].load(blobs, "obs")
    B[1].load(snapshot_fixture("withMarkers"))
    o = OracleDoc()
    o.load_v1(blobs, "obs")
    tail = _remote_tail(o, 3, 100, 40, 10, ["client-1", "client-2"])
    for m in tail:
        B[0].applyMsg(m)
    B.flush()
    first = (B.dump_segments(0), B.dump_segments(1))
    B.rewind()
    B.replay_resident()
    assert (B.dump_segments(0), B.dump_segments(1)) == first
    _same(B, 0, o, "after rewind + resident replay")
