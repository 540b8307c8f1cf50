"""GPU parity of the SnapshotLegacy summary (snapshotlegacy.ts:122-259).

The engine's legacy writer (mtb_summarize_legacy) reads the replayed tree and emits the header / body
chunks at the MSN; the oracle's writer is pinned byte-exact by the reference's 6 snapshots/legacy files
(tests/test_oracle.py).  Bar: blobs and ISummaryTreeWithStats byte-equal to the oracle after collaborative
replay — the 30 reference logs at every 8th group and at the end, synthetic logs in both length modes, a
small chunk size (header + body), and a catch-up messages blob.
"""
import pytest

from helpers import msg_from_compact, replay_fixtures

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chunk", [0, 64])
def test_reference_logs_legacy_summaries(chunk):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    fx = replay_fixtures()
    B = MergeTreeBatch(len(fx), chunk_size=chunk)
    oracles = []
    for i, (_, d) in enumerate(fx):
        B[i].insertTextLocal(0, d["initialText"])
        B[i].startOrUpdateCollaboration("A")
        o = OracleDoc(chunk_size=chunk)
        o.insert_text_local(0, d["initialText"])
        o.start_collab("A")
        oracles.append(o)
    ngroups = len(fx[0][1]["groups"])
    for g in range(ngroups):
        for i, (_, d) in enumerate(fx):
            for m in d["groups"][g]["msgs"]:
                B[i].applyMsg(msg_from_compact(m))
                oracles[i].apply_msg(msg_from_compact(m))
        if g % 8 == 7 or g == ngroups - 1:
            B.flush()
            for i, (name, _) in enumerate(fx):
                gb, gs = B.summarize_legacy(i)
                osum = oracles[i].summarize_legacy()
                assert [list(x) for x in gb] == osum["blobs"], f"{name} group {g}: legacy blobs differ"
                assert gs == osum["summary"], f"{name} group {g}: summary tree differs"


@pytest.mark.parametrize("new_mode", [False, True])
def test_synthetic_logs_legacy_summary_with_catch_up(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    from pyloggen import LogBatch, make_cfg
    from helpers import records_to_msgs
    cfg = make_cfg(seed=91 + int(new_mode), n_ops=1200, new_length_calc=new_mode)
    lb = LogBatch(cfg, 0, 16)
    props = lb.props_json()
    B = MergeTreeBatch(lb.n, new_length_calc=new_mode, chunk_size=500)
    oracles, tails = [], []
    for i in range(lb.n):
        tb = lb.doc_text_bytes(i)
        il = lb.docs[i].initial_len
        msgs = records_to_msgs(lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb, props, lb.client_ids(i))
        B[i].insertTextLocal(0, tb[: il * 2].decode("utf-16-le"))
        B[i].startOrUpdateCollaboration("obs")
        o = OracleDoc(new_length_calc=new_mode, chunk_size=500)
        o.insert_text_local(0, tb[: il * 2].decode("utf-16-le"))
        o.start_collab("obs")
        for m in msgs:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
        msn = msgs[-1]["minimumSequenceNumber"]
        tails.append([dict(m, minimumSequenceNumber=msn) for m in msgs if m["sequenceNumber"] > msn])
    B.flush()
    for i in range(lb.n):
        gb, gs = B.summarize_legacy(i, catchup=tails[i])
        osum = oracles[i].summarize_legacy(catchup=tails[i])
        assert [list(x) for x in gb] == osum["blobs"], f"doc {i}: legacy blobs differ"
        assert gs == osum["summary"], f"doc {i}: summary tree differs"
        assert any(p == "catchupOps" for p, _ in gb) == bool(tails[i])


@pytest.mark.parametrize("chunk", [0, 300])
def test_reference_logs_legacy_catch_up_rewriting(chunk):
    """MTB_BATCH_CATCHUP: the engine keeps messagesSinceMSNChange and rewrites lagging messages from the
    kernel's delta entries; the legacy summary (header/body + catchupOps) equals the oracle's, whose
    rewriting replays to the golden final text (tests/test_oracle.py)."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    fx = replay_fixtures()
    B = MergeTreeBatch(len(fx), chunk_size=chunk, catch_up=True)
    oracles = []
    for i, (_, d) in enumerate(fx):
        B[i].insertTextLocal(0, d["initialText"])
        B[i].startOrUpdateCollaboration("A")
        o = OracleDoc(chunk_size=chunk)
        o.insert_text_local(0, d["initialText"])
        o.start_collab("A")
        o.enable_catch_up()
        oracles.append(o)
    ngroups = len(fx[0][1]["groups"])
    for g in range(ngroups):
        for i, (_, d) in enumerate(fx):
            for m in d["groups"][g]["msgs"]:
                B[i].applyMsg(msg_from_compact(m))
                oracles[i].apply_msg(msg_from_compact(m))
        if g % 16 == 15:
            B.flush()
            for i, (name, _) in enumerate(fx):
                gb, gs = B.summarize_legacy(i)
                osum = oracles[i].summarize_legacy()
                assert [list(x) for x in gb] == osum["blobs"], f"{name} group {g}: legacy + catch-up blobs differ"
                assert gs == osum["summary"], f"{name} group {g}"


@pytest.mark.parametrize("new_mode", [False, True])
def test_synthetic_logs_catch_up_rewriting(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    from pyloggen import LogBatch, make_cfg
    from helpers import records_to_msgs
    cfg = make_cfg(seed=123 + int(new_mode), n_ops=1000, new_length_calc=new_mode)
    lb = LogBatch(cfg, 0, 16)
    props = lb.props_json()
    B = MergeTreeBatch(lb.n, new_length_calc=new_mode, catch_up=True)
    oracles = []
    for i in range(lb.n):
        tb = lb.doc_text_bytes(i)
        il = lb.docs[i].initial_len
        B[i].insertTextLocal(0, tb[: il * 2].decode("utf-16-le"))
        B[i].startOrUpdateCollaboration("obs")
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, tb[: il * 2].decode("utf-16-le"))
        o.start_collab("obs")
        o.enable_catch_up()
        for m in records_to_msgs(lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb, props, lb.client_ids(i)):
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
    B.flush()
    for i in range(lb.n):
        gb, gs = B.summarize_legacy(i)
        osum = oracles[i].summarize_legacy()
        assert [list(x) for x in gb] == osum["blobs"], f"doc {i}: legacy + catch-up blobs differ"
        assert any(p == "catchupOps" for p, _ in gb)


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations",
                                  "withIntervals"])
def test_reference_legacy_summaries_load_on_the_engine(name):
    """Client.load of the reference's snapshots/legacy files (toLatestVersion, snapshotChunks.ts:151-199):
    the engine's text and dump equal the oracle that loaded them, and its SnapshotLegacy gives the fixture
    bytes back."""
    from fluidframework_amd import MergeTreeBatch
    from helpers import snapshot_fixture
    from pyoracle import OracleDoc
    blobs = snapshot_fixture(name, "legacy")
    o = OracleDoc()
    o.load_v1(blobs, "loader")
    B = MergeTreeBatch(1)
    assert B[0].loadSequence(dict(blobs), "loader") == []
    assert B.text(0) == o.get_text()
    assert B.dump_segments(0) == o.dump_segments()
    gb, _ = B.summarize_legacy(0, 0, 0)
    assert [list(x) for x in gb] == blobs


@pytest.mark.parametrize("g", [16, 40])
@pytest.mark.parametrize("chunk", [0, 300])
def test_legacy_load_with_catch_up_continues_the_reference_logs(g, chunk):
    """SharedSegmentSequence.loadCore on the engine (sequence.ts:568-610) for the 30 reference logs: a legacy
    summary (with its catch-up blob) taken by the oracle after g groups is loaded by loadSequence (body
    chunks on the GPU, catch-up messages validated against the window and replayed), then the rest of the
    log: the golden text after every later group, dumps equal to the oracle that loaded the same summary,
    and a legacy summary equal to that oracle's at the end."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    fx = replay_fixtures()
    B = MergeTreeBatch(len(fx), chunk_size=chunk, catch_up=True)
    loaded = []
    for i, (_, d) in enumerate(fx):
        src = OracleDoc(chunk_size=chunk)
        src.insert_text_local(0, d["initialText"])
        src.start_collab("A")
        src.enable_catch_up()
        for grp in d["groups"][:g]:
            for m in grp["msgs"]:
                src.apply_msg(msg_from_compact(m))
        blobs = src.summarize_legacy()["blobs"]
        o = OracleDoc(chunk_size=chunk)
        o.enable_catch_up()
        o.apply_catch_up(o.load_v1(blobs, "loader"))
        assert B[i].loadSequence(blobs, "loader"), "the logs leave messages above the MSN"
        loaded.append(o)
    B.flush()
    for i, o in enumerate(loaded):
        assert B.dump_segments(i) == o.dump_segments(), f"{fx[i][0]}: dump after catch-up"
    ngroups = len(fx[0][1]["groups"])
    for grp_i in range(g, ngroups):
        for i, (_, d) in enumerate(fx):
            for m in d["groups"][grp_i]["msgs"]:
                B[i].applyMsg(msg_from_compact(m))
                loaded[i].apply_msg(msg_from_compact(m))
        B.flush()
        for i, (name, d) in enumerate(fx):
            assert B.text(i) == d["groups"][grp_i]["resultText"], f"{name} group {grp_i}"
    for i, (name, _) in enumerate(fx):
        assert B.dump_segments(i) == loaded[i].dump_segments(), name
        gb, gs = B.summarize_legacy(i)
        assert [list(x) for x in gb] == loaded[i].summarize_legacy()["blobs"], name


def test_catch_up_rewriting_kat_on_the_engine():
    """The hand-derived catch-up known answer of tests/test_oracle.py::test_catch_up_rewriting_kat on the engine:
    a lagging rewrite's ops name its deleted keys (old order) then its own (segmentPropertiesManager.ts:107-154,
    kernel entries tagged MTB_DELTA_OLD carry the sets before it); a lagging incr's NaN values never coalesce."""
    import json
    from fluidframework_amd import MergeTreeBatch
    B = MergeTreeBatch(1, catch_up=True)
    B[0].insertTextLocal(0, "abcdef", {"s": "x", "m": 0})
    B[0].startOrUpdateCollaboration("A")
    msg = dict(type="op", minimumSequenceNumber=0, referenceSequenceNumber=0)
    B[0].applyMsg(dict(msg, clientId="c1", sequenceNumber=1, contents={"type": 0, "pos1": 0, "seg": "zz"}))
    B[0].applyMsg(dict(msg, clientId="c2", sequenceNumber=2, contents={
        "type": 2, "pos1": 2, "pos2": 4, "props": {"n": 1, "m": 0}, "combiningOp": {"name": "rewrite"}}))
    B[0].applyMsg(dict(msg, clientId="c3", sequenceNumber=3, contents={
        "type": 2, "pos1": 0, "pos2": 4, "props": {"m": 1}, "combiningOp": {"name": "incr"}}))
    B.flush()
    gb, _ = B.summarize_legacy(0)
    cu = json.loads(dict(gb)["catchupOps"])
    assert [m["contents"] for m in cu] == [
        {"type": 0, "pos1": 0, "seg": "zz"},
        {"pos1": 4, "pos2": 6, "props": {"s": None, "m": 0, "n": 1}, "type": 2},
        {"ops": [{"pos1": 2, "pos2": 4, "props": {"m": None}, "type": 2},
                 {"pos1": 4, "pos2": 6, "props": {"m": None}, "type": 2}], "type": 3}]
    assert list(cu[1]["contents"]["props"]) == ["s", "m", "n"]


@pytest.mark.parametrize("new_mode", [False, True])
def test_catch_up_rewriting_of_rewrite_and_incr_annotates(new_mode):
    """Lagging rewrite and incr annotates in the catch-up blob (createOpsFromDelta, sequence.ts:120-172): the
    engine's legacy summary with catch-up equals the oracle's mid-log; loadSequence of it on the engine equals
    the oracle that loaded the same blobs (dump), and both continue to the same text and dump."""
    from fluidframework_amd import MergeTreeBatch
    from helpers import make_incr_log
    from pyoracle import OracleDoc
    n, cut = 12, 450
    logs = [make_incr_log(300 + i, 700, lag=24, new_mode=new_mode, p_incr=0.15 if i % 2 else 0.0, p_rewrite=0.2)
            for i in range(n)]
    B = MergeTreeBatch(n, new_length_calc=new_mode, catch_up=True)
    oracles = []
    for i, (init, msgs) in enumerate(logs):
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("A")
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, init)
        o.start_collab("A")
        o.enable_catch_up()
        for m in msgs[:cut]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
    B.flush()
    L = MergeTreeBatch(n, new_length_calc=new_mode)
    loaded = []
    for i, o in enumerate(oracles):
        gb, gs = B.summarize_legacy(i)
        osum = o.summarize_legacy()
        assert [list(x) for x in gb] == osum["blobs"], f"doc {i}: legacy + catch-up blobs differ"
        r = OracleDoc(new_length_calc=new_mode)
        r.apply_catch_up(r.load_v1(osum["blobs"], "loader"))
        assert L[i].loadSequence(osum["blobs"], "loader")
        loaded.append(r)
    L.flush()
    for i, r in enumerate(loaded):
        assert L.dump_segments(i) == r.dump_segments(), f"doc {i}: dump after catch-up"
        for m in logs[i][1][cut:]:
            L[i].applyMsg(m)
            r.apply_msg(m)
    L.flush()
    for i, r in enumerate(loaded):
        assert L.text(i) == r.get_text() and L.dump_segments(i) == r.dump_segments(), f"doc {i}"


def test_catch_up_validation_follows_the_moving_window_on_the_engine():
    """loadSequence reads the collab window again for every catch-up message (sequence.ts:578-585): after a
    message raised minSeq to its MSN, a later message with a lower MSN is "Invalid catchup operations in
    snapshot" -- on the Python drop-in as on the oracle."""
    import json
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from pyoracle import OracleDoc, OracleError
    from test_oracle import _msn_backwards
    name, d = replay_fixtures()[3]
    src = OracleDoc()
    src.insert_text_local(0, d["initialText"])
    src.start_collab("A")
    src.enable_catch_up()
    for grp in d["groups"][:20]:
        for m in grp["msgs"]:
            src.apply_msg(msg_from_compact(m))
    blobs = src.summarize_legacy()["blobs"]
    known = {"header", "body"}
    k = next(i for i, (p, _) in enumerate(blobs) if p not in known)
    bad = [list(b) for b in blobs]
    bad[k][1] = json.dumps(_msn_backwards(json.loads(blobs[k][1])))
    o = OracleDoc()
    with pytest.raises(OracleError, match="Invalid catchup"):
        o.apply_catch_up(o.load_v1(bad, "loader"))
    B = MergeTreeBatch(1, catch_up=True)
    with pytest.raises(MergeTreeError, match="Invalid catchup operations in snapshot"):
        B[0].loadSequence(bad, "loader")


@pytest.mark.parametrize("new_mode", [False, True])
def test_catch_up_with_marker_relative_positions(new_mode):
    """SharedString's default configuration (SnapshotLegacy + messagesSinceMSNChange) with annotateMarker and
    other marker-relative ops (opBuilder.ts:25-43): a message that saw everything before it is stored verbatim,
    relative positions and all, a lagging one is rewritten from its delta to absolute positions
    (sequence.ts:704-726, createOpsFromDelta :120-172).  Mid-log legacy summaries with catch-up blobs equal the
    oracle's byte for byte; loadSequence of them on the engine (relative positions resolved against the loaded
    markers) equals the oracle that loaded the same blobs, and both continue to the same text and dump."""
    import json
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from helpers import make_marker_log
    from pyoracle import OracleDoc, OracleError
    n, cut = 10, 500
    logs = [make_marker_log(700 + i, 900, n_clients=3 + i % 3, lag=4 + 3 * i, new_mode=new_mode) for i in range(n)]
    B = MergeTreeBatch(n, new_length_calc=new_mode, catch_up=True)
    oracles = []
    for i, (init, msgs) in enumerate(logs):
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("A")
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, init)
        o.start_collab("A")
        o.enable_catch_up()
        for m in msgs[:cut]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
    B.flush()
    L = MergeTreeBatch(n, new_length_calc=new_mode)
    loaded, verbatim_rel, refused = {}, 0, 0
    for i, o in enumerate(oracles):
        gb, gs = B.summarize_legacy(i)
        osum = o.summarize_legacy()
        assert [list(x) for x in gb] == osum["blobs"], f"doc {i}: legacy + catch-up blobs differ"
        cu = json.loads(dict(osum["blobs"])["catchupOps"])
        verbatim_rel += sum(1 for m in cu if "relativePos1" in json.dumps(m["contents"]))
        r = OracleDoc(new_length_calc=new_mode)
        try:
            r.apply_catch_up(r.load_v1(osum["blobs"], "loader"))
        except OracleError as e:
            # a verbatim message naming a marker removed at or below the MSN: the summary has no such marker
            # (posFromRelativePos -1); both refuse the document
            assert "names no marker" in str(e)
            with pytest.raises(MergeTreeError, match="names no marker"):
                L[i].loadSequence(osum["blobs"], "loader")
            refused += 1
            continue
        assert L[i].loadSequence(osum["blobs"], "loader")
        loaded[i] = r
    assert verbatim_rel > 0, "the catch-up blobs hold no relative-position message"
    assert len(loaded) >= n // 2, f"{refused} of {n} documents refused"
    L.flush()
    for i, r in loaded.items():
        assert L.dump_segments(i) == r.dump_segments(), f"doc {i}: dump after catch-up"
        for m in logs[i][1][cut:]:
            try:
                r.apply_msg(m)
            except OracleError as e:  # (as above: a marker the loaded summary does not hold)
                assert "names no marker" in str(e)
                with pytest.raises(MergeTreeError, match="names no marker"):
                    L[i].applyMsg(m)
                break
            L[i].applyMsg(m)
    L.flush()
    for i, r in loaded.items():
        assert L.text(i) == r.get_text() and L.dump_segments(i) == r.dump_segments(), f"doc {i}"


@pytest.mark.parametrize("new_mode", [False, True])
def test_catch_up_rewriting_with_irregular_values_and_consensus(new_mode):
    """Lagging annotates whose values matchProperties does not compare as an equivalence (helpers.make_props_log:
    primitives against objects, nested nulls, remote consensus values) in the catch-up blob: createOpsFromDelta
    (sequence.ts:120-172) merges neighbouring ranges with matchProperties(lastAnnotate.props, props) over the
    segments' own values (a consensus value, its `value` member undefined, never matches).  Blobs equal to the
    oracle's; loadSequence continues to the same text and dump."""
    from fluidframework_amd import MergeTreeBatch
    from helpers import make_props_log
    from pyoracle import OracleDoc
    n, cut = 10, 450
    logs = [make_props_log(600 + i + 20 * int(new_mode), 700, lag=24, new_mode=new_mode) for i in range(n)]
    B = MergeTreeBatch(n, new_length_calc=new_mode, catch_up=True)
    oracles = []
    for i, (init, msgs) in enumerate(logs):
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("A")
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, init)
        o.start_collab("A")
        o.enable_catch_up()
        for m in msgs[:cut]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
    B.flush()
    L = MergeTreeBatch(n, new_length_calc=new_mode)
    loaded = []
    for i, o in enumerate(oracles):
        gb, gs = B.summarize_legacy(i)
        osum = o.summarize_legacy()
        assert [list(x) for x in gb] == osum["blobs"], f"doc {i}: legacy + catch-up blobs differ"
        r = OracleDoc(new_length_calc=new_mode)
        r.apply_catch_up(r.load_v1(osum["blobs"], "loader"))
        assert L[i].loadSequence(osum["blobs"], "loader")
        loaded.append(r)
    L.flush()
    for i, r in enumerate(loaded):
        assert L.dump_segments(i) == r.dump_segments(), f"doc {i}: dump after catch-up"
        for m in logs[i][1][cut:]:
            L[i].applyMsg(m)
            r.apply_msg(m)
    L.flush()
    for i, r in enumerate(loaded):
        assert L.text(i) == r.get_text() and L.dump_segments(i) == r.dump_segments(), f"doc {i}"
