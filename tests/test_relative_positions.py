"""Marker-relative positions (IRelativePosition, ops.ts:77-92; getValidOpRange client.ts:527-547;
posFromRelativePos mergeTree.ts:1371-1395; idToSegment :549 filled by insertSegments :1658-1663 and every
blockUpdate :2392 -> addNodeReferences :296-306).

CPU side: the oracle restatement (known answers built from the reference's rules — the reference commits
no relative-position golden data, so these are oracle-defined, parity unpinned beyond code reading) and the
host packer's pack-time rejections (no GPU needed).  The engine's parity against the oracle is in
tests/test_gpu_relpos.py."""
import pytest

from helpers import make_marker_log


def _msg(cid, seq, ref, msn, op):
    return {"clientId": cid, "sequenceNumber": seq, "referenceSequenceNumber": ref, "minimumSequenceNumber": msn,
            "type": "op", "contents": op}


def _doc(new_mode=False):
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode, verify=True)
    o.insert_text_local(0, "hello world")
    o.start_collab("obs")
    return o


def test_relative_insert_before_and_after_marker():
    o = _doc()
    o.apply_msg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 5, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m"}}}))
    o.apply_msg(_msg("a", 2, 1, 0, {"type": 0, "relativePos1": {"id": "m", "before": True}, "seg": "<"}))
    o.apply_msg(_msg("a", 3, 2, 0, {"type": 0, "relativePos1": {"id": "m"}, "seg": ">"}))
    o.apply_msg(_msg("a", 4, 3, 0, {"type": 0, "relativePos1": {"id": "m", "offset": 2}, "seg": "!"}))
    o.apply_msg(_msg("a", 5, 4, 0, {"type": 0, "relativePos1": {"id": "m", "before": True, "offset": 3}, "seg": "^"}))
    # the marker (not in the text) sits after "hello<" (position 6): after it + 2 is before "w", before it - 3 is 3
    assert o.get_text() == "hel^lo<> !world"


def test_annotate_marker_touches_only_the_marker():
    o = _doc()
    o.apply_msg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 3, "seg": {"marker": {"refType": 0}, "props": {"markerId": "q"}}}))
    # createAnnotateMarkerOp (opBuilder.ts:25-43)
    o.apply_msg(_msg("b", 2, 1, 0, {"type": 2, "relativePos1": {"id": "q", "before": True}, "relativePos2": {"id": "q"},
                                    "props": {"state": "open"}}))
    rows = [e for e in o.map_range() if e["segment"].get("properties", {}).get("state") == "open"]
    assert len(rows) == 1 and rows[0]["segment"]["type"] == "Marker" and rows[0]["pos"] == 3


def test_relative_position_in_a_lagging_view():
    o = _doc()
    o.apply_msg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 0, "seg": "AAAA"}))
    o.apply_msg(_msg("a", 2, 1, 0, {"type": 0, "pos1": 9, "seg": {"marker": {}, "props": {"markerId": "z"}}}))
    # client b has not seen seq 1: the marker is at 5 in its view (getPosition sums (refSeq, client) lengths)
    assert o.pos_from_relative({"id": "z", "before": True}, 0, 0) == 9  # observer id 0 = local view at currentSeq
    o.add_client("b")
    b = 2  # short id of "b" (obs 0, a 1)
    assert o.pos_from_relative({"id": "z", "before": True}, 1, b) == 9
    assert o.pos_from_relative({"id": "z", "before": True}, 0, b) == 5
    o.apply_msg(_msg("b", 3, 0, 0, {"type": 0, "relativePos1": {"id": "z"}, "seg": "#"}))
    # "after" adds marker.cachedLength even where the marker is invisible (b has not seen seq 2), so the
    # insert lands one character into " world" in b's view
    assert o.get_text() == "AAAAhello #world"


def test_unknown_and_falsy_ids_resolve_to_minus_one():
    o = _doc()
    o.apply_msg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 2, "seg": {"marker": {}, "props": {"markerId": 7}}}))
    assert o.pos_from_relative({"id": "nope"}, 1, 0) == -1
    assert o.pos_from_relative({"id": ""}, 1, 0) == -1
    assert o.pos_from_relative({"id": "7"}, 1, 0) == -1  # Map identity: the number 7 is not the string "7"
    assert o.pos_from_relative({"id": 7}, 1, 0) == 3
    from pyoracle import OracleError
    with pytest.raises(OracleError, match="names no marker"):
        o.apply_msg(_msg("a", 2, 1, 0, {"type": 1, "relativePos1": {"id": "nope"}, "pos2": 4}))


def test_unlinked_marker_position_is_zero():
    """zamboni unlinks a removed marker (segment.parent = undefined, zamboni.ts:146); idToSegment keeps it
    and getPosition of a parentless node is 0 (mergeTree.ts:768-785)."""
    o = _doc()
    o.apply_msg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 6, "seg": {"marker": {}, "props": {"markerId": "u"}}}))
    o.apply_msg(_msg("a", 2, 1, 1, {"type": 1, "pos1": 6, "pos2": 7}))
    assert o.pos_from_relative({"id": "u", "before": True}, 2, 0) == 6
    for s in range(3, 8):  # advance the MSN past the removal; zamboni scours the marker's block
        o.apply_msg(_msg("a", s, s - 1, s - 1, {"type": 2, "pos1": 0, "pos2": 1, "props": {"x": s}}))
    assert o.pos_from_relative({"id": "u", "before": True}, 7, 0) == 0
    assert o.pos_from_relative({"id": "u", "offset": 1}, 7, 0) == 2


def test_duplicate_ids_follow_block_update():
    """Two markers with one id: insertSegments maps the newer one; any later blockUpdate of the older
    one's block maps the older one back (children in order, last wins) — observable through relative
    positions.  Oracle-defined; the engine's marker kernel re-maps the same way (tests/test_gpu_relpos.py)."""
    o = _doc()
    o.apply_msg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 2, "seg": {"marker": {}, "props": {"markerId": "d"}}}))
    o.apply_msg(_msg("a", 2, 1, 0, {"type": 0, "pos1": 9, "seg": {"marker": {}, "props": {"markerId": "d"}}}))
    # the tree is one leaf block: inserting the second marker ran blockUpdate over it, mapping the first
    # marker (child order) and then the second
    assert o.pos_from_relative({"id": "d", "before": True}, 2, 0) == 9


@pytest.mark.parametrize("new_mode", [False, True])
def test_marker_log_generator_replays_on_a_fresh_oracle(new_mode):
    from pyoracle import OracleDoc
    init, msgs = make_marker_log(11, 600, new_mode=new_mode)
    n_rel = sum(1 for m in msgs if any(k.startswith("relativePos") for k in m["contents"]))
    assert n_rel > 100
    o = OracleDoc(new_length_calc=new_mode, verify=True)
    o.insert_text_local(0, init)
    o.start_collab("obs")
    for m in msgs:
        o.apply_msg(m)
    assert o.get_length() > 0


def test_host_rejects_unresolvable_relative_positions_at_pack_time():
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    B = MergeTreeBatch(1)
    B[0].startOrUpdateCollaboration("A")
    mk = {"type": 0, "pos1": 0, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m1"}}}
    B[0].applyMsg(_msg("B", 1, 0, 0, mk))
    with pytest.raises(MergeTreeError, match="names no marker"):
        B[0].applyMsg(_msg("B", 2, 1, 0, {"type": 0, "relativePos1": {"id": "m2"}, "seg": "x"}))
    with pytest.raises(MergeTreeError, match="non-integer"):
        B[0].applyMsg(_msg("B", 2, 1, 0, {"type": 0, "relativePos1": {"id": "m1", "offset": 1.5}, "seg": "x"}))
    B[0].applyMsg(_msg("B", 2, 1, 0, {"type": 0, "relativePos1": {"id": "m1", "before": True}, "seg": "x"}))
    import struct
    ob, n, _ = B.export_pending(0)
    t, fl, c, seq, ref, msn, p1, p2, pay, pr = struct.unpack_from("<BBHIIIIIII", ob, 32 * (n - 1))
    assert fl & 0x20 and p1 & 0x80000000  # MTB_F_RELPOS: pos1 names a descriptor
    t, fl, c, seq, ref, msn, p1, p2, pay, pr = struct.unpack_from("<BBHIIIIIII", ob, 0)
    assert fl & 0x02 and pay == 1  # the marker carries its id ordinal + 1
    # a reused id: the marker and live kernels re-map it at blockUpdate time, so relative positions naming
    # it pack, in an observer's document and in a live client's, before or after its first local op
    B[0].applyMsg(_msg("B", 3, 2, 0, mk))
    rm = {"type": 1, "relativePos1": {"id": "m1", "before": True}, "relativePos2": {"id": "m1"}}
    B[0].applyMsg(_msg("B", 4, 3, 0, rm))
    B[0].insertSegmentLocal(0, "x")
    L = MergeTreeBatch(1)
    L[0].startOrUpdateCollaboration("A")
    L[0].applyMsg(_msg("B", 1, 0, 0, mk))
    L[0].applyMsg(_msg("B", 2, 1, 0, mk))
    L[0].insertSegmentLocal(0, "x")
    L[0].applyMsg(_msg("B", 3, 2, 0, rm))
    # catch-up batches take relative positions too (round 5: tests/test_gpu_legacy.py)
    C = MergeTreeBatch(1, catch_up=True)
    C[0].startOrUpdateCollaboration("A")
    C[0].applyMsg(_msg("B", 1, 0, 0, mk))
    C[0].applyMsg(_msg("B", 2, 1, 0, {"type": 0, "relativePos1": {"id": "m1"}, "seg": "x"}))
    with pytest.raises(MergeTreeError, match="names no marker"):
        C[0].applyMsg(_msg("B", 3, 2, 0, {"type": 0, "relativePos1": {"id": "zz"}, "seg": "x"}))


def test_annotate_may_not_change_a_marker_id():
    """annotateRange's assert 0x5ad (mergeTree.ts:1912-1918): props naming markerId must carry each annotated
    marker's own id (JS ===): the same primitive passes, another value / null / an object fails, a marker
    without an id fails, text segments are not checked."""
    from pyoracle import OracleError

    def doc_with_markers():
        o = _doc()
        o.apply_msg(_msg("a", 1, 0, 0, {"type": 0, "pos1": 2, "seg": {"marker": {"refType": 1}, "props": {"markerId": "k"}}}))
        o.apply_msg(_msg("a", 2, 1, 0, {"type": 0, "pos1": 8, "seg": {"marker": {"refType": 1}}}))
        return o

    o = doc_with_markers()
    o.apply_msg(_msg("b", 3, 2, 0, {"type": 2, "pos1": 2, "pos2": 3, "props": {"markerId": "k", "x": 1}}))
    o.apply_msg(_msg("b", 4, 3, 0, {"type": 2, "pos1": 4, "pos2": 7, "props": {"markerId": "text-ok"}}))
    assert o.pos_from_relative({"id": "k", "before": True}, 4, 0) == 2
    for props, at in (({"markerId": "z"}, 2), ({"markerId": None}, 2), ({"markerId": {"k": 1}}, 2), ({"markerId": "k"}, 8)):
        o = doc_with_markers()
        with pytest.raises(OracleError, match="0x5ad"):
            o.apply_msg(_msg("b", 3, 2, 0, {"type": 2, "pos1": at, "pos2": at + 1, "props": props}))


@pytest.mark.parametrize("new_mode", [False, True])
def test_duplicate_id_log_generator_replays_on_a_fresh_oracle(new_mode):
    """make_marker_log(dup_ids=...) streams (reused ids, markerId annotates, rewrites dropping ids) replay."""
    from pyoracle import OracleDoc
    init, msgs = make_marker_log(21, 500, new_mode=new_mode, dup_ids=3)
    assert sum(1 for m in msgs if "markerId" in (m["contents"].get("props") or {}) and m["contents"]["type"] == 2) > 10
    o = OracleDoc(new_length_calc=new_mode, verify=True)
    o.insert_text_local(0, init)
    o.start_collab("obs")
    for m in msgs:
        o.apply_msg(m)
