"""GPU parity of marker-relative positions (IRelativePosition, ops.ts:77-92): getValidOpRange
(client.ts:527-547) resolving relativePos1/2 with posFromRelativePos (mergeTree.ts:1371-1395) in the op's
(refSeq, client) view, over idToSegment (:549) filled by marker inserts (:1658-1663), summary loads
(reloadFromSegments -> blockUpdate :296-306; body inserts) — resolved on the GPU (the kernel's rel_pos walks
the marker's ancestors, getPosition :768-785).

Bar: bit-exact against the oracle (canonical segment dump, text, state digest, SnapshotV1) on
* generated logs (tests/helpers.make_marker_log): markers with unique ids, annotateMarker ops
  (opBuilder.ts:25-43), inserts / removes / annotates with relative positions (before / offset), lagging
  views, removed and zamboni-unlinked markers; both length modes, two flushes;
* the reference's withMarkers SnapshotV1 fixture (markers "marker0", "marker70", ... with markerId in
  header and body chunks) loaded, then remote ops relative to its markers;
* a relative position whose marker is a removed header marker (never mapped: posFromRelativePos -1) fails
  its document with the engine's "relative position" error, the other documents replay.
"""
import random

import pytest

from helpers import first_diff, make_marker_log, snapshot_fixture

pytestmark = pytest.mark.gpu


def _same(B, i, o, what):
    gd, od = B.dump_segments(i), o.dump_segments()
    assert gd == od, f"{what}: segment dump differs: {first_diff(gd, od)}"
    assert B.text(i) == o.get_text(), f"{what}: text differs"
    assert B.digests(i, 1)[0] == o.digest(), f"{what}: digest differs"


@pytest.mark.parametrize("new_mode", [False, True])
def test_marker_relative_logs(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    logs = [make_marker_log(100 + s, 900, n_clients=3 + s % 4, lag=8 + 6 * s, new_mode=new_mode) for s in range(10)]
    B = MergeTreeBatch(len(logs), new_length_calc=new_mode)
    orc = []
    for i, (init, _) in enumerate(logs):
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("obs")
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, init)
        o.start_collab("obs")
        orc.append(o)
    for part in (slice(0, 450), slice(450, None)):
        for i, (_, msgs) in enumerate(logs):
            for m in msgs[part]:
                B[i].applyMsg(m)
                orc[i].apply_msg(m)
        st = B.replay()
        assert st["errors"] == 0, st
        for i, o in enumerate(orc):
            _same(B, i, o, f"log {i} {part}")
    for i, o in enumerate(orc):
        gb, gs = B.summarize_v1(i)
        assert [list(x) for x in gb] == o.summarize_v1()["blobs"], f"log {i}: SnapshotV1 differs"


def test_relative_ops_on_the_reference_withMarkers_summary():
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    blobs = snapshot_fixture("withMarkers")
    rng = random.Random(5)
    o = OracleDoc()
    o.load_v1(blobs, "obs")
    ids = [f"marker{70 * k}" for k in range(0, 140)]
    ids = [m for m in ids if o.pos_from_relative({"id": m, "before": True}, 0, 0) >= 0]
    assert len(ids) > 100  # header and body markers
    B = MergeTreeBatch(1)
    B[0].load(dict(blobs), "obs")
    msgs, seq = [], 0
    for k in range(300):
        seq += 1
        cid = rng.choice(["a", "b", "c"])
        ref = max(0, seq - 1 - rng.randint(0, 10))
        mid = rng.choice(ids)
        r = rng.random()
        if r < 0.4:
            op = {"type": 2, "relativePos1": {"id": mid, "before": True}, "relativePos2": {"id": mid},
                  "props": {"Properties": {"Bold": rng.random() < 0.5}}}
        elif r < 0.8:
            op = {"type": 0, "relativePos1": {"id": mid, "offset": rng.randint(0, 4)}, "seg": rng.choice(["x", "yz", "\n"])}
        else:
            op = {"type": 1, "relativePos1": {"id": mid}, "relativePos2": {"id": mid, "offset": rng.randint(1, 3)}}
        m = {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,
             "minimumSequenceNumber": max(0, seq - 12), "type": "op", "contents": op}
        o.apply_msg(m)
        B[0].applyMsg(m)
        if k % 100 == 99:
            st = B.replay()
            assert st["errors"] == 0, st
            _same(B, 0, o, f"after {k + 1} ops")


def test_unmapped_marker_fails_its_document_only():
    """A removed header marker is never mapped (blockUpdate maps live markers only): the reference's
    posFromRelativePos gives -1, which the engine (and the oracle) rejects for that document."""
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from pyoracle import OracleDoc, OracleError
    summary_src = OracleDoc()
    summary_src.insert_text_local(0, "abcdef")
    summary_src.insert_marker_local(3, 1, {"markerId": "gone"})
    summary_src.insert_marker_local(1, 1, {"markerId": "live"})
    summary_src.start_collab("w")
    summary_src.add_client("x")
    summary_src.apply_msg({"clientId": "x", "sequenceNumber": 1, "referenceSequenceNumber": 0,
                           "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 1, "pos1": 4, "pos2": 5}})
    blobs = summary_src.summarize_v1()["blobs"]
    bad = {"clientId": "y", "sequenceNumber": 2, "referenceSequenceNumber": 1, "minimumSequenceNumber": 0, "type": "op",
           "contents": {"type": 0, "relativePos1": {"id": "gone"}, "seg": "!"}}
    good = dict(bad, contents={"type": 0, "relativePos1": {"id": "live"}, "seg": "!"})
    o = OracleDoc()
    o.load_v1(blobs, "obs")
    with pytest.raises(OracleError, match="names no marker"):
        o.apply_msg(bad)
    B = MergeTreeBatch(2)
    for i in range(2):
        B[i].load([tuple(x) for x in blobs], "obs")
    B[0].applyMsg(bad)
    B[1].applyMsg(good)
    with pytest.raises(MergeTreeError, match="relative position"):
        B.replay()
    o2 = OracleDoc()
    o2.load_v1(blobs, "obs")
    o2.apply_msg(good)
    assert B.text(1) == o2.get_text()


def test_relative_positions_in_a_live_client_batch():
    """A live client's own marker (local insert, pending then acked) named by remote relative ops: the
    live-client kernel carries the marker map too."""
    import json
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    o = OracleDoc()
    o.insert_text_local(0, "hello world")
    o.start_collab("me")
    B = MergeTreeBatch(1)
    B[0].insertTextLocal(0, "hello world")
    B[0].startOrUpdateCollaboration("me")
    op = o.insert_local_op(5, {"marker": {"refType": 1}, "props": {"markerId": "L"}})
    op = json.loads(op) if isinstance(op, str) else op
    B[0].applyLocalOp(op)
    msgs = [
        {"clientId": "x", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0, "type": "op",
         "contents": {"type": 0, "pos1": 0, "seg": "AB"}},
        {"clientId": "me", "sequenceNumber": 2, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0, "type": "op",
         "contents": op},
        {"clientId": "x", "sequenceNumber": 3, "referenceSequenceNumber": 1, "minimumSequenceNumber": 0, "type": "op",
         "contents": {"type": 0, "relativePos1": {"id": "L", "before": True}, "seg": "<"}},
        {"clientId": "y", "sequenceNumber": 4, "referenceSequenceNumber": 3, "minimumSequenceNumber": 1, "type": "op",
         "contents": {"type": 2, "relativePos1": {"id": "L", "before": True}, "relativePos2": {"id": "L"},
                      "props": {"seen": True}}},
    ]
    for k, m in enumerate(msgs):
        o.apply_msg(m)
        B[0].applyMsg(m)
        B.replay()
        _same(B, 0, o, f"after message {k + 1}")


def test_annotate_marker_of_a_live_client():
    """Client.annotateMarker (client.ts:190-197): a live client's local annotate whose positions are
    relative to a marker, resolved in its own view; its keys stay pending against a concurrent remote
    annotate until the ack; then a remote relative op and a reconnect-free continuation."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=True)
    o.insert_text_local(0, "hello world")
    o.start_collab("me")
    B = MergeTreeBatch(1, new_length_calc=True)
    c = B[0]
    c.insertTextLocal(0, "hello world")
    c.startOrUpdateCollaboration("me")
    steps = [
        ("msg", {"clientId": "x", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
                 "type": "op", "contents": {"type": 0, "pos1": 5, "seg": {"marker": {"refType": 1},
                                                                          "props": {"markerId": "p1"}}}}),
        ("mark", ("p1", {"color": "red", "n": 1})),
        ("msg", {"clientId": "x", "sequenceNumber": 2, "referenceSequenceNumber": 1, "minimumSequenceNumber": 0,
                 "type": "op", "contents": {"type": 2, "relativePos1": {"id": "p1", "before": True},
                                            "relativePos2": {"id": "p1"}, "props": {"color": "blue", "w": 2}}}),
        ("ack", 3),
        ("msg", {"clientId": "x", "sequenceNumber": 4, "referenceSequenceNumber": 3, "minimumSequenceNumber": 1,
                 "type": "op", "contents": {"type": 2, "relativePos1": {"id": "p1", "before": True},
                                            "relativePos2": {"id": "p1", "offset": 3}, "props": {"color": "green"}}}),
    ]
    last = None
    for kind, x in steps:
        if kind == "msg":
            o.apply_msg(x)
            c.applyMsg(x)
        elif kind == "mark":
            last = c.annotateMarker(x[0], x[1])
            assert o.local_op_json(last) == last
        else:
            ack = {"clientId": "me", "sequenceNumber": x, "referenceSequenceNumber": 1, "minimumSequenceNumber": 1,
                   "type": "op", "contents": last}
            o.apply_msg(ack)
            c.applyMsg(ack)
        B.replay()
        _same(B, 0, o, f"after {kind}")
    segs = [e["segment"] for e in B.map_range(0) if e["segment"].get("type") == "Marker"]
    assert segs[0]["properties"]["color"] == "green" and segs[0]["properties"]["n"] == 1


def test_get_text_range_counts_markers():
    """TestClient.getText(start, end) (testClient.ts:185, MergeTreeTextHelper.ts:20-81): positions count
    markers (length 1), which add no text."""
    from fluidframework_amd import MergeTreeBatch
    B = MergeTreeBatch(1)
    c = B[0]
    c.insertTextLocal(0, "hello world")
    c.startOrUpdateCollaboration("me")
    c.applyMsg({"clientId": "x", "sequenceNumber": 1, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
                "type": "op", "contents": {"type": 0, "pos1": 5, "seg": {"marker": {"refType": 1}}}})
    assert c.getText() == "hello world"
    assert c.getText(3, 8) == "lo w"  # l o [marker] ' ' w
    assert c.getText(5, 6) == ""
    assert c.getText(6) == " world"
    assert c.getText(None, 2) == "he"


def test_test_client_helpers_reference_applymsg_kat():
    """TestClient helpers (testClient.ts:224-327) driving client.applyMsg.spec.ts-style steps: remote insert,
    marker, annotate and remove messages made by makeOpMessage."""
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.client import TestClient
    B = MergeTreeBatch(1)
    c = B[0]
    assert isinstance(c, TestClient)
    c.insertTextLocal(0, "hello world")
    c.startOrUpdateCollaboration("me")
    c.insertTextRemote(0, "ab", None, 1, 0, "a")
    c.insertMarkerRemote(2, {"refType": 1}, {"markerId": "m"}, 2, 1, "b")
    c.annotateRangeRemote(0, 2, {"x": 1}, 3, 2, "a")
    c.removeRangeRemote(3, 9, 4, 3, "b")
    assert c.getText() == "abworld"
    assert c.getText(0, 3) == "ab"
    props = [e["segment"].get("properties") for e in B.map_range(0, 0, 2)]
    assert props == [{"x": 1}]


@pytest.mark.parametrize("new_mode", [False, True])
def test_reused_marker_ids_follow_block_update(new_mode):
    """Marker ids reused across markers (make_marker_log(dup_ids=...)): which marker an id names is decided
    by the last blockUpdate of a leaf block holding one of them (mergeTree.ts:2392 -> addNodeReferences
    :296-306; insertingWalk :1780-1846, split :1858-1871, markRangeRemoved's post-order :2019-2026,
    zamboni.ts:55/:103), with annotates naming markerId (assert 0x5ad) and rewrites dropping ids.  The
    marker kernel's re-mapping (DSF_MKDUP) against the oracle: dumps, text, digests, SnapshotV1."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    logs = [make_marker_log(300 + s, 800, n_clients=3 + s % 3, lag=4 + 5 * s, new_mode=new_mode, dup_ids=2 + s % 4)
            for s in range(12)]
    B = MergeTreeBatch(len(logs), new_length_calc=new_mode)
    orc = []
    for i, (init, _) in enumerate(logs):
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("obs")
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, init)
        o.start_collab("obs")
        orc.append(o)
    for part in (slice(0, 300), slice(300, None)):
        for i, (_, msgs) in enumerate(logs):
            for m in msgs[part]:
                B[i].applyMsg(m)
                orc[i].apply_msg(m)
        st = B.replay()
        assert st["errors"] == 0, st
        for i, o in enumerate(orc):
            _same(B, i, o, f"log {i} {part}")
    for i, o in enumerate(orc):
        gb, gs = B.summarize_v1(i)
        assert [list(x) for x in gb] == o.summarize_v1()["blobs"], f"log {i}: SnapshotV1 differs"


def test_reused_id_kat_and_marker_id_assert_on_the_engine():
    """test_relative_positions.py's duplicate-id KAT (the newer marker's insert re-maps the older one too,
    child order: the last wins) and assert 0x5ad (an annotate changing a marker's id) fail / pass per
    document on the engine exactly as on the oracle."""
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from pyoracle import OracleDoc, OracleError

    def msg(cid, seq, ref, op):
        return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": 0,
                "type": "op", "contents": op}

    mk = lambda pos, mid: {"type": 0, "pos1": pos, "seg": {"marker": {"refType": 1}, "props": {"markerId": mid}}}
    kat = [msg("a", 1, 0, mk(2, "d")), msg("a", 2, 1, mk(9, "d")),
           msg("b", 3, 2, {"type": 0, "relativePos1": {"id": "d", "before": True}, "seg": "<"})]
    assert_log = [msg("a", 1, 0, mk(2, "k")), msg("b", 2, 1, {"type": 2, "pos1": 2, "pos2": 3, "props": {"markerId": "z"}})]
    ok_log = [msg("a", 1, 0, mk(2, "k")), msg("b", 2, 1, {"type": 2, "pos1": 1, "pos2": 4, "props": {"markerId": "k"}}),
              msg("b", 3, 2, {"type": 0, "relativePos1": {"id": "k"}, "seg": ">"})]
    B = MergeTreeBatch(3)
    for i, log in enumerate((kat, assert_log, ok_log)):
        B[i].insertTextLocal(0, "hello world")
        B[i].startOrUpdateCollaboration("obs")
        for m in log:
            B[i].applyMsg(m)
    with pytest.raises(MergeTreeError, match="0x5ad"):
        B.replay()
    for i, log in ((0, kat), (2, ok_log)):
        o = OracleDoc()
        o.insert_text_local(0, "hello world")
        o.start_collab("obs")
        for m in log:
            o.apply_msg(m)
        _same(B, i, o, f"doc {i}")
    assert B.text(0) == "hello wo<rld"  # inserted before the newer marker "d" (position 9)
    o = OracleDoc()
    o.insert_text_local(0, "hello world")
    o.start_collab("obs")
    o.apply_msg(assert_log[0])
    with pytest.raises(OracleError, match="0x5ad"):
        o.apply_msg(assert_log[1])


def test_loaded_summary_with_reused_marker_ids():
    """A SnapshotV1 header and body holding several markers per id (reloadFromSegments' blockUpdate maps the
    last live one; body inserts re-map through insertingWalk), then marker-relative ops naming them."""
    import random as _r
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    rng = _r.Random(9)
    src = OracleDoc(chunk_size=40)
    src.insert_text_local(0, "x" * 120)
    for k in range(24):
        src.insert_marker_local(rng.randint(0, src.get_length()), 1, {"markerId": f"d{k % 3}"})
    src.start_collab("w")
    blobs = src.summarize_v1()["blobs"]
    assert any("body_" in p for p, _ in blobs)
    gen = OracleDoc(chunk_size=40)
    gen.load_v1(blobs, "gen")
    msgs, seq = [], 0
    while len(msgs) < 300:
        seq += 1
        cid = rng.choice(["a", "b", "c"])
        ref = max(0, seq - 1 - rng.randint(0, 6))
        mid = f"d{rng.randrange(3)}"
        r = rng.random()
        if r < 0.3:
            op = {"type": 0, "pos1": rng.randint(0, gen.remote_length(ref, 0)),
                  "seg": {"marker": {"refType": 1}, "props": {"markerId": mid}}}
        elif r < 0.7:
            op = {"type": 0, "relativePos1": {"id": mid, "before": rng.random() < 0.5}, "seg": rng.choice(["y", "zz"])}
        else:
            op = {"type": 1, "relativePos1": {"id": mid, "before": True}, "relativePos2": {"id": mid, "offset": 1}}
        m = {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref,
             "minimumSequenceNumber": max(0, seq - 8), "type": "op", "contents": op}
        probe = OracleDoc(chunk_size=40)  # keep only ops valid in the sender's view
        probe.load_v1(blobs, "gen")
        try:
            for x in msgs + [m]:
                probe.apply_msg(x)
        except Exception:
            seq -= 1
            continue
        gen.apply_msg(m)
        msgs.append(m)
    o = OracleDoc(chunk_size=40)
    o.load_v1(blobs, "obs")
    B = MergeTreeBatch(1, chunk_size=40)
    B[0].load([tuple(x) for x in blobs], "obs")
    for m in msgs:
        B[0].applyMsg(m)
        o.apply_msg(m)
    st = B.replay()
    assert st["errors"] == 0, st
    _same(B, 0, o, "loaded reused ids")
