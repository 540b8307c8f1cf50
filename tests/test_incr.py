"""combiningOp "incr" annotates (segmentPropertiesManager.ts:145-147 calls combine(combiningOp, previousValue,
undefined, seq), properties.ts:24-69): restated known answers on the oracle, and the engine's pack-time
checks (CPU; the engine's replay parity is tests/test_gpu_incr.py).

JS semantics pinned here (oracle-defined: the reference commits no incr data; each case is the JS expression
the reference evaluates):
* a number / boolean / absent value + undefined is NaN; JSON.stringify writes it as null;
* NaN !== NaN, so matchProperties never matches a set holding NaN -- not even a copy of itself (split halves
  never coalesce again, zamboni and SnapshotV1 alike);
* a string value gets "undefined" appended; minValue (when truthy) replaces a smaller string;
* a remote incr modifies keys with pending local updates too (shouldModifyKey returns true for a combiningOp).
"""
import json

import pytest

from test_reference_kats import msg


def _doc(text="abcdefgh", new_mode=False, observer="obs"):
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode, verify=True)
    o.insert_text_local(0, text)
    o.start_collab(observer)
    return o


def _rows(o):
    return [json.loads(line) for line in o.dump_segments().splitlines()[1:]]


def test_incr_number_and_absent_become_nan():
    o = _doc()
    o.apply_msg(msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 4, "props": {"n": 1, "s": "x"}}))
    o.apply_msg(msg("a", 2, 1, {"type": 2, "pos1": 2, "pos2": 6, "props": {"n": 5}, "combiningOp": {"name": "incr"}}))
    rows = [(r[2], r[7]) for r in _rows(o)]
    assert rows == [("ab", {"n": 1, "s": "x"}), ("cd", {"n": None, "s": "x"}), ("ef", {"n": None}), ("gh", None)]


def test_incr_string_concatenates_and_min_value():
    o = _doc()
    o.apply_msg(msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 2, "props": {"s": "abc"}}))
    o.apply_msg(msg("a", 2, 1, {"type": 2, "pos1": 0, "pos2": 1, "props": {"s": 1}, "combiningOp": {"name": "incr"}}))
    o.apply_msg(msg("a", 3, 2, {"type": 2, "pos1": 1, "pos2": 2, "props": {"s": 1},
                                "combiningOp": {"name": "incr", "minValue": "zz"}}))
    rows = [(r[2], r[7]) for r in _rows(o)]
    assert rows[:2] == [("a", {"s": "abcundefined"}), ("b", {"s": "zz"})]


def test_nan_sets_never_coalesce():
    """Two neighbours that each hold NaN (even split halves of one annotated segment) stay apart through
    zamboni and in SnapshotV1, where equal numeric values would merge."""
    o = _doc("abcd")
    o.apply_msg(msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 4, "props": {"n": 1}, "combiningOp": {"name": "incr"}}))
    o.apply_msg(msg("a", 2, 1, {"type": 0, "pos1": 2, "seg": "X"}))
    o.apply_msg(msg("a", 3, 2, {"type": 1, "pos1": 2, "pos2": 3}, msn=3))
    o.apply_msg(msg("a", 4, 3, {"type": 0, "pos1": 0, "seg": "Y"}, msn=4))  # zamboni past every seq
    texts = [r[2] for r in _rows(o) if r[5] == -1]
    assert "ab" in texts and "cd" in texts, texts
    segs = json.loads(o.summarize_v1()["blobs"][0][1])["segments"]
    assert {"text": "ab", "props": {"n": None}} in segs and {"text": "cd", "props": {"n": None}} in segs
    # the same with a plain numeric value coalesces
    p = _doc("abcd")
    p.apply_msg(msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 4, "props": {"n": 1}}))
    p.apply_msg(msg("a", 2, 1, {"type": 0, "pos1": 2, "seg": "X"}))
    p.apply_msg(msg("a", 3, 2, {"type": 1, "pos1": 2, "pos2": 3}, msn=3))
    p.apply_msg(msg("a", 4, 3, {"type": 0, "pos1": 0, "seg": "Y"}, msn=4))
    assert "abcd" in [r[2] for r in _rows(p)]


def test_remote_incr_modifies_pending_local_keys():
    """shouldModifyKey (segmentPropertiesManager.ts:95-106) is true for a combiningOp: a remote incr changes a
    key the local client has a pending annotate on; a plain remote annotate does not."""
    o = _doc("abcdef", observer="me")
    op = o.annotate_local_op(1, 4, {"n": 7})
    o.apply_msg(msg("x", 1, 0, {"type": 2, "pos1": 0, "pos2": 6, "props": {"n": 2}}))
    assert [r[7] for r in _rows(o)][1] == {"n": 7}
    o.apply_msg(msg("x", 2, 1, {"type": 2, "pos1": 0, "pos2": 6, "props": {"n": 1}, "combiningOp": {"name": "incr"}}))
    assert [r[7] for r in _rows(o)] == [{"n": None}, {"n": None}, {"n": None}]
    o.apply_msg(msg("me", 3, 0, op))


def test_host_incr_packing():
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    B = MergeTreeBatch(1)
    B[0].startOrUpdateCollaboration("obs")
    B[0].applyMsg(msg("a", 1, 0, {"type": 0, "pos1": 0, "seg": "abc"}))
    B[0].applyMsg(msg("a", 2, 1, {"type": 2, "pos1": 0, "pos2": 2, "props": {"n": 1}, "combiningOp": {"name": "incr"}}))
    B[0].applyMsg(msg("a", 3, 2, {"type": 2, "pos1": 0, "pos2": 2, "props": {"n": 1},
                                  "combiningOp": {"name": "incr", "defaultValue": 4, "minValue": 2}}))
    B[0].applyMsg(msg("a", 4, 3, {"type": 2, "pos1": 0, "pos2": 2, "props": {"n": 1},
                                  "combiningOp": {"name": "incr", "defaultValue": "x"}}))  # (a string result)
    with pytest.raises(MergeTreeError, match="object defaultValue"):
        B[0].applyMsg(msg("a", 5, 4, {"type": 2, "pos1": 0, "pos2": 2, "props": {"n": 1},
                                      "combiningOp": {"name": "incr", "defaultValue": {"a": 1}}}))
    B[0].applyMsg(msg("a", 5, 4, {"type": 2, "pos1": 0, "pos2": 2, "props": {"n": 1},
                                  "combiningOp": {"name": "consensus"}}))
    import struct
    ob, n, _ = B.export_pending(0)
    t, fl = struct.unpack_from("<BB", ob, 32)
    assert t == 2 and fl & 0x0C == 0x08  # MTB_F_INCR
    t, fl = struct.unpack_from("<BB", ob, 32 * 4)
    assert t == 2 and fl & 0x0C == 0x0C  # MTB_F_CONSENSUS
