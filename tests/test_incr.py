"""combiningOp "incr" annotates (segmentPropertiesManager.ts:145-147 calls combine(combiningOp, previousValue,
undefined, seq), properties.ts:24-69): restated known answers on the oracle, and the engine's pack-time
checks (CPU; the engine's replay parity is tests/test_gpu_incr.py).

JS semantics pinned here (oracle-defined: the reference commits no incr data; each case is the JS expression
the reference evaluates):
* a number / boolean / absent value + undefined is NaN; JSON.stringify writes it as null;
* NaN !== NaN, so matchProperties never matches a set holding NaN -- not even a copy of itself (split halves
  never coalesce again, zamboni and SnapshotV1 alike);
* a string value gets "undefined" appended; minValue (when truthy) replaces a smaller string;
* an object or array value (or defaultValue) is String()-converted first ("[object Object]", join(",")), and an
  object minValue compares as its string form;
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


def test_incr_object_and_array_values_concatenate_their_string_form():
    """_currentValue += undefined on an object is String(obj) + "undefined" ("[object Object]undefined"), on an array
    Array.prototype.join(",") (undefined / null elements empty, nested arrays joined, objects "[object Object]")
    + "undefined"; an object or array defaultValue concatenates the same way; an object minValue compares as its
    string form and, when larger, replaces the result with the object itself."""
    o = _doc()
    o.apply_msg(msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 4,
                                "props": {"o": {"x": 1}, "a": [1, None, "s", [2, 3], {"y": 1}, True, 1.5]}}))
    o.apply_msg(msg("a", 2, 1, {"type": 2, "pos1": 0, "pos2": 2, "props": {"o": 1, "a": 1},
                                "combiningOp": {"name": "incr"}}))
    o.apply_msg(msg("a", 3, 2, {"type": 2, "pos1": 4, "pos2": 6, "props": {"o": 1, "a": 1},
                                "combiningOp": {"name": "incr", "defaultValue": [7, [8]]}}))
    o.apply_msg(msg("a", 4, 3, {"type": 2, "pos1": 6, "pos2": 7, "props": {"s": 1},
                                "combiningOp": {"name": "incr", "defaultValue": "A", "minValue": {"z": 1}}}))
    o.apply_msg(msg("a", 5, 4, {"type": 2, "pos1": 7, "pos2": 8, "props": {"s": 1},
                                "combiningOp": {"name": "incr", "defaultValue": "b", "minValue": {"z": 1}}}))
    rows = [(r[2], r[7]) for r in _rows(o)]
    assert rows == [
        ("ab", {"o": "[object Object]undefined", "a": "1,,s,2,3,[object Object],true,1.5undefined"}),
        ("cd", {"o": {"x": 1}, "a": [1, None, "s", [2, 3], {"y": 1}, True, 1.5]}),
        ("ef", {"o": "7,8undefined", "a": "7,8undefined"}),
        ("g", {"s": {"z": 1}}),  # "Aundefined" < "[object Object]": the minValue object itself
        ("h", {"s": "bundefined"}),
    ], rows


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
    B[0].applyMsg(msg("a", 5, 4, {"type": 2, "pos1": 0, "pos2": 2, "props": {"n": 1},
                                  "combiningOp": {"name": "incr", "defaultValue": {"a": 1}, "minValue": [1]}}))
    B[0].applyMsg(msg("a", 6, 5, {"type": 2, "pos1": 0, "pos2": 2, "props": {"n": 1},
                                  "combiningOp": {"name": "consensus"}}))
    import struct
    ob, n, _ = B.export_pending(0)
    t, fl = struct.unpack_from("<BB", ob, 32)
    assert t == 2 and fl & 0x0C == 0x08  # MTB_F_INCR
    t, fl = struct.unpack_from("<BB", ob, 32 * 5)
    assert t == 2 and fl & 0x0C == 0x0C  # MTB_F_CONSENSUS


def test_incr_tables_are_per_document():
    """An incr annotate's result table covers the values its own document can hold (DocVals in mtb_host.cpp), so
    one document's many distinct values under a key neither enlarge nor refuse another document's incr on it;
    the refusal (more than 4096 concatenating values under the key in one document) stays with that document."""
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    B = MergeTreeBatch(2)
    for i in range(2):
        B[i].startOrUpdateCollaboration("obs")
        B[i].applyMsg(msg("a", 1, 0, {"type": 0, "pos1": 0, "seg": "abcdef"}))
    seq = 2
    for j in range(4200):  # document 0: 4,200 distinct strings under "author"
        B[0].applyMsg(msg("a", seq, seq - 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"author": f"name{j}"}}))
        seq += 1
    B[1].applyMsg(msg("a", 2, 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"author": "me"}}))
    B[1].applyMsg(msg("a", 3, 2, {"type": 2, "pos1": 0, "pos2": 6, "props": {"author": 1},
                                  "combiningOp": {"name": "incr"}}))  # document 1 holds one string: accepted
    with pytest.raises(MergeTreeError, match="4096"):
        B[0].applyMsg(msg("a", seq, seq - 1, {"type": 2, "pos1": 0, "pos2": 6, "props": {"author": 1},
                                              "combiningOp": {"name": "incr"}}))
    B[1].applyMsg(msg("a", 4, 3, {"type": 2, "pos1": 0, "pos2": 6, "props": {"author": 1},
                                  "combiningOp": {"name": "incr"}}))  # (and still accepted after the refusal)
