"""Known answers for matchProperties (merge-tree/src/properties.ts:71-96) where it is no equivalence, and for
remote "consensus" annotates (properties.ts:46-62 via segmentPropertiesManager.ts:145-147).  Each expectation
is derived by hand from those lines (the reference commits no data for them):

matchProperties(a, b) walks the keys of a; b[key] undefined fails; typeof b[key] === "object" (objects, arrays
and null) recurses with (a[key], b[key]); anything else compares b[key] !== a[key].  The recursion sees
primitives through Object.keys (numbers and booleans have none, a string has its indices), so
* {k: 5} matches {k: {}} and {k: "ab"} matches {k: {"0": "a", "1": "b"}}, but not the reverse;
* {k: {x: 0}} matches {k: {x: null}} (both falsy) but not the reverse (null !== 0);
* zamboni (zamboni.ts:151-177) and SnapshotV1 (snapshotV1.ts:238-251) compare each segment with the run's
  head, so [{k: "a"}, {k: {"0": "a"}}, {k: "a"}] becomes one segment although its neighbours do not match.

A remote consensus annotate computes combine(op, previous, undefined, seq) per key: no previous value and no
defaultValue gives a fresh {value: undefined, seq} (JSON {"seq": seq}; its undefined member makes every
matchProperties with it as b false, so two such segments never coalesce live, yet do after a summary round
trip); a present value stays; a defaultValue object whose seq is -1 gets the op's seq.

Each case: (name, initial text, messages, expected rows [text, props] of the live segments after the log).
Messages advance the MSN to the last seq so that zamboni has run over every segment."""
from test_reference_kats import msg


def _ins(c, seq, ref, pos, text, props, msn=0):
    return msg(c, seq, ref, {"type": 0, "pos1": pos, "seg": {"text": text, "props": props}}, msn=msn)


def _tick(seq):
    """ops that advance the MSN past every earlier seq (zamboni over every segment): insert "#" at 0, remove it,
    then insert "." at 0 (it stays, and joins a following segment without properties)"""
    return [msg("z", seq, seq - 1, {"type": 0, "pos1": 0, "seg": "#"}, msn=seq - 1),
            msg("z", seq + 1, seq, {"type": 1, "pos1": 0, "pos2": 1}, msn=seq + 1),
            msg("z", seq + 2, seq + 1, {"type": 0, "pos1": 0, "seg": "."}, msn=seq + 2)]


def _three(values):
    out = []
    pos = 0
    for i, v in enumerate(values):
        t = "abcdef"[2 * i:2 * i + 2]
        out.append(_ins("a", i + 1, i, pos, t, {"k": v}))
        pos += 2
    return out + _tick(len(values) + 1)


CASES = [
    ("primitive head, object next: coalesce", "",
     _three([5, {}]), [[".", None], ["abcd", {"k": 5}]]),
    ("object head, primitive next: apart", "",
     _three([{}, 5]), [[".", None], ["ab", {"k": {}}], ["cd", {"k": 5}]]),
    ("string head, index object next: coalesce", "",
     _three(["ab", {"0": "a", "1": "b"}]), [[".", None], ["abcd", {"k": "ab"}]]),
    ("index object head, string next: apart", "",
     _three([{"0": "a", "1": "b"}, "ab"]), [[".", None], ["ab", {"k": {"0": "a", "1": "b"}}], ["cd", {"k": "ab"}]]),
    ("nested zero head, nested null next: coalesce", "",
     _three([{"x": 0}, {"x": None}]), [[".", None], ["abcd", {"k": {"x": 0}}]]),
    ("nested null head, nested zero next: apart", "",
     _three([{"x": None}, {"x": 0}]), [[".", None], ["ab", {"k": {"x": None}}], ["cd", {"k": {"x": 0}}]]),
    ("nested nulls: coalesce", "",
     _three([{"x": None}, {"x": None}]), [[".", None], ["abcd", {"k": {"x": None}}]]),
    ("run head decides, not the neighbour", "",
     _three(["a", {"0": "a"}, "a"]), [[".", None], ["abcdef", {"k": "a"}]]),
    ("empty array against a number", "",
     _three([7, []]), [[".", None], ["abcd", {"k": 7}]]),
    ("consensus: fresh values stay apart, present values stay", "abcdef",
     [msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 2, "props": {"k": 1}}),
      msg("a", 2, 1, {"type": 2, "pos1": 0, "pos2": 4, "props": {"k": 9}, "combiningOp": {"name": "consensus"}}),
      msg("b", 3, 2, {"type": 0, "pos1": 3, "seg": "X"}),
      msg("b", 4, 3, {"type": 1, "pos1": 3, "pos2": 4})] + _tick(5),
     [[".", None], ["ab", {"k": 1}], ["c", {"k": {"seq": 2}}], ["d", {"k": {"seq": 2}}], ["ef", None]]),
    ("consensus: a defaultValue object with seq -1 takes the op's seq", "abcdef",
     [msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 6, "props": {"k": 1, "j": None},
                      "combiningOp": {"name": "consensus", "defaultValue": {"seq": -1, "v": [1]}}}),
      msg("b", 2, 1, {"type": 0, "pos1": 3, "seg": "X"}),
      msg("b", 3, 2, {"type": 1, "pos1": 3, "pos2": 4})] + _tick(4),
     [[".", None], ["abcdef", {"k": {"seq": 1, "v": [1]}, "j": {"seq": 1, "v": [1]}}]]),
    ("consensus: a primitive defaultValue", "abcd",
     [msg("a", 1, 0, {"type": 2, "pos1": 1, "pos2": 3, "props": {"k": 1},
                      "combiningOp": {"name": "consensus", "defaultValue": "d"}})] + _tick(2),
     [[".a", None], ["bc", {"k": "d"}], ["d", None]]),  # (the tick's "." joins the unannotated "a")
    # incr makes NaN (JSON null): matchProperties(NaN, {}) recurses into (NaN, {}) whose key lists are both empty,
    # so a NaN head takes an empty-object (or empty-array) neighbour; the reverse compares {} !== NaN
    ("NaN head, empty object next: coalesce", "",
     [_ins("a", 1, 0, 0, "ab", {"k": 5}), _ins("a", 2, 1, 2, "cd", {"k": {}}),
      msg("a", 3, 2, {"type": 2, "pos1": 0, "pos2": 2, "props": {"k": 1}, "combiningOp": {"name": "incr"}})] + _tick(4),
     [[".", None], ["abcd", {"k": None}]]),
    ("empty array head, NaN next: apart", "",
     [_ins("a", 1, 0, 0, "ab", {"k": []}), _ins("a", 2, 1, 2, "cd", {"k": 5}),
      msg("a", 3, 2, {"type": 2, "pos1": 2, "pos2": 4, "props": {"k": 1}, "combiningOp": {"name": "incr"}})] + _tick(4),
     [[".", None], ["ab", {"k": []}], ["cd", {"k": None}]]),
    ("NaN head, non-empty object next: apart", "",
     [_ins("a", 1, 0, 0, "ab", {"k": 5}), _ins("a", 2, 1, 2, "cd", {"k": {"x": 1}}),
      msg("a", 3, 2, {"type": 2, "pos1": 0, "pos2": 2, "props": {"k": 1}, "combiningOp": {"name": "incr"}})] + _tick(4),
     [[".", None], ["ab", {"k": None}], ["cd", {"k": {"x": 1}}]]),
]

# (name, initial text, messages, error substring): the reference mutates a shared object or throws
REFUSED = [
    ("consensus over an object value whose seq is -1", "abcd",
     [_ins("a", 1, 0, 0, "xy", {"k": {"seq": -1}}),
      msg("a", 2, 1, {"type": 2, "pos1": 0, "pos2": 3, "props": {"k": 1}, "combiningOp": {"name": "consensus"}})],
     "seq is -1"),
]

# (name, initial text, messages, error substring): the reference itself throws at the last message (JS TypeError)
THROWS = [
    ("consensus with a null defaultValue over a segment lacking the key", "abcd",
     [msg("a", 1, 0, {"type": 2, "pos1": 0, "pos2": 3, "props": {"k": 1},
                      "combiningOp": {"name": "consensus", "defaultValue": None}})],
     "TypeError"),
]


def rows(dump):
    """[text, props] of the unremoved segments of a canonical dump"""
    import json
    out = []
    for line in dump.splitlines()[1:]:
        r = json.loads(line)
        if r[5] == -1:
            out.append([r[2], r[7]])
    return out
