"""The reference KATs of tests/test_reference_kats.py on the GPU engine: expected texts / lengths / segment
orders / child counts from the reference tests, and the canonical segment dump equal to the oracle fed the
same calls.  All-remote cases use an observer; cases with local ops use live clients (detached tombstones of
createClientsAtInitialState via mtb_detached_op_json, zamboniSegments / packParent via mtb_maintenance).

* mergeTree.markRangeRemoved.spec.ts:114-154 and the passive observer of :156-227;
* partialLength.spec.ts:39-297, the remote-client tables (a view's length is the sum of mapRange over it);
* mergeTree.annotate.spec.ts:529-575 (a remote annotate; a later split copies its properties);
* client.applyMsg.spec.ts:415-493 ("CB", "ab", #9703 "ayzXd" in new length mode), three live clients;
* mergeTree.insertingWalk.spec.ts:285-356 (the segment order ["G","F","E","(D)",...,"x","0"]);
* mergeTree.zamboni.spec.ts:22-80 (lengths and child counts around zamboniSegments / packParent).
"""
import pytest

from test_reference_kats import msg, passive_observer_race_msgs

pytestmark = pytest.mark.gpu


def _run(initial, observer, msgs, clients=(), new_mode=False):
    """(engine batch, oracle) after the same messages."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    B = MergeTreeBatch(1, new_length_calc=new_mode)
    B.init_doc(0, initial, observer)
    o = OracleDoc(new_length_calc=new_mode, verify=True)
    if initial:
        o.insert_text_local(0, initial)
    o.start_collab(observer)
    for c in clients:
        B.add_client(0, c)
        o.add_client(c)
    for m in msgs:
        B[0].applyMsg(m)
        o.apply_msg(m)
    B.replay()
    assert B.dump_segments(0) == o.dump_segments()
    return B, o


def _hello(extra):
    return [msg("local", i + 1, i, {"type": 0, "pos1": i, "seg": ch}) for i, ch in enumerate("hello world")] + extra


def test_remote_remove_then_remote_insert():
    B, _ = _run("", "A", _hello([msg("remote2", 12, 11, {"type": 1, "pos1": 0, "pos2": 11}),
                                 msg("remote", 13, 11, {"type": 0, "pos1": 0, "seg": "text"})]))
    assert B.text(0) == "text"


def test_remote_insert_then_remote_remove():
    B, _ = _run("", "A", _hello([msg("remote", 12, 11, {"type": 0, "pos1": 0, "seg": "text"}),
                                 msg("remote2", 13, 11, {"type": 1, "pos1": 0, "pos2": 11})]))
    assert B.text(0) == "text"


@pytest.mark.parametrize("new_mode", [False, True])
def test_passive_observer_race(new_mode):
    B, _ = _run("", "3", passive_observer_race_msgs(), new_mode=new_mode)
    assert B.text(0) == "cX"


def _view_len(B, ref, client):
    """The document's length in (ref, client)'s view: mapRange over all of it visits exactly the segments
    with a non-zero length there (nodeMap, mergeTree.ts:2556-2558), each with its whole cachedLength."""
    return sum(e["segment"]["cachedLength"] for e in B.map_range(0, 0, -1, ref, client))


def _partial(msgs):
    return _run("hello world!", "obs", msgs, clients=("c17", "c18", "c19"))


def test_partial_lengths_tables():
    B, o = _partial([])
    assert _view_len(B, 0, "c17") == 12
    for w in ("c17", "c18"):
        B, o = _partial([msg(w, 1, 0, {"type": 0, "pos1": 0, "seg": "more "})])
        assert _view_len(B, 1, "c17") == 17 and _view_len(B, 1, "c18") == 17
        B, o = _partial([msg(w, 1, 0, {"type": 1, "pos1": 0, "pos2": 12})])
        assert _view_len(B, 1, "c17") == 0 and _view_len(B, 1, "c18") == 0
    B, o = _partial([msg(w, k + 1, k, {"type": 0, "pos1": 0, "seg": t})
                     for k, (w, t) in enumerate([("c17", "1"), ("c18", "2"), ("c17", "3"), ("c18", "4")])])
    assert _view_len(B, 4, "c17") == 16 and _view_len(B, 4, "c18") == 16
    B, o = _partial([msg("c17", i + 1, i, {"type": 0, "pos1": 0, "seg": "a"}) for i in range(100)])
    assert _view_len(B, 100, "c17") == 112 and _view_len(B, 100, "c18") == 112
    for s in range(1, 101):  # every view of the window, against the oracle's (leaf-sum checked) lengths
        for c in ("c17", "c18"):
            assert _view_len(B, s, c) == o.remote_length(s, o.client_ids().index(c))
    B, o = _partial([msg("c18", 1, 0, {"type": 1, "pos1": 0, "pos2": 10}),
                     msg("c19", 2, 0, {"type": 1, "pos1": 0, "pos2": 10})])
    assert _view_len(B, 1, "c17") == 2
    B, o = _partial([msg("c17", 1, 0, {"type": 1, "pos1": 0, "pos2": 10}),
                     msg("c18", 2, 0, {"type": 1, "pos1": 0, "pos2": 10})])
    assert _view_len(B, 1, "c17") == 2 and _view_len(B, 1, "c18") == 2


def test_annotate_remote_first_split_copies_props():
    props = {"propertySource": "remote", "remoteProperty": 1}
    B, o = _run("hello world!", "local", [
        msg("remote", 1, 0, {"type": 0, "pos1": 3, "seg": {"marker": {"refType": 1}}}),
        msg("remote", 2, 1, {"type": 2, "pos1": 1, "pos2": 5, "props": props}),
        msg("other", 3, 2, {"type": 0, "pos1": 2, "seg": "Z"})])
    segs = [e["segment"] for e in B.map_range(0)]
    assert [s.get("text") for s in segs[:4]] == ["h", "e", "Z", "l"]
    assert segs[1].get("properties") == props and segs[3].get("properties") == props
    assert B.text(0) == "heZllo world!"


# ------------------------------------------------------------------ KATs with local ops / detached tombstones
# (VERDICT r03 weak 1): the reference's literals asserted on the engine, every client a live client of one
# batch; each engine client is paired with an oracle client fed the same calls (canonical dumps equal too).

class _Pair:
    """One reference TestClient: engine document k of batch B and an oracle client, built like
    createClientsAtInitialState (testClientLogger.ts:51-78): insertTextLocal(0, state), then every "-"
    removed locally while detached, then startOrUpdateCollaboration(id)."""

    def __init__(self, B, k, cid, state, new_mode):
        from pyoracle import OracleDoc
        self.B, self.k, self.id = B, k, cid
        self.c = B[k]
        self.o = OracleDoc(new_length_calc=new_mode, verify=True)
        if state:
            self.c.insertTextLocal(0, state)
            self.o.insert_text_local(0, state)
        text = state
        while "-" in text:
            i = text.index("-")
            self.c.removeRangeLocal(i, i + 1)
            self.o.remove_local(i, i + 1)
            text = text[:i] + text[i + 1:]
        self.c.startOrUpdateCollaboration(cid)
        self.o.start_collab(cid)

    def local(self, kind, *args):
        """insertTextLocal / removeRangeLocal on both; returns the op (the engine's equals the oracle's)."""
        if kind == "insert":
            op, oop = self.c.insertTextLocal(*args), self.o.insert_local_op(*args)
        else:
            op, oop = self.c.removeRangeLocal(*args), self.o.remove_local_op(*args)
        assert op == oop, (op, oop)
        return op

    def make(self, op, seq):
        """TestClient.makeOpMessage(op, seq) (testClient.ts:303-327): refSeq = the client's currentSeq."""
        return msg(self.id, seq, self.o.current_seq, op)

    def apply(self, m):
        self.c.applyMsg(m)
        self.o.apply_msg(m)

    @property
    def current_seq(self):
        return self.o.current_seq

    def check(self, text):
        assert self.B.dump_segments(self.k) == self.o.dump_segments(), f"client {self.id}: dump"
        assert self.c.getText() == self.o.get_text() == text, (self.id, self.c.getText(), self.o.get_text(), text)
        assert self.c.getCurrentSeq() == self.o.current_seq


def _clients(state, ids=("A", "B", "C"), new_mode=False):
    from fluidframework_amd import MergeTreeBatch
    B = MergeTreeBatch(len(ids), new_length_calc=new_mode)
    return B, {cid: _Pair(B, k, cid, state, new_mode) for k, cid in enumerate(ids)}


@pytest.mark.parametrize("new_mode", [False, True])
def test_applymsg_remote_remove_before_conflicting_insert(new_mode):
    """client.applyMsg.spec.ts:415-438 ("Remote Remove before conflicting insert") -> "CB"."""
    B, c = _clients("Z", new_mode=new_mode)
    seq = 0
    seq += 1
    op1 = c["B"].make(c["B"].local("remove", 0, 1), seq)
    seq += 1
    op2 = c["B"].make(c["B"].local("insert", 0, "B"), seq)
    c["C"].apply(op1)
    seq += 1
    op3 = c["C"].make(c["C"].local("insert", 0, "C"), seq)
    c["A"].apply(op1)
    c["B"].apply(op1)
    for m in (op2, op3):
        for p in c.values():
            p.apply(m)
    for p in c.values():
        p.check("CB")


@pytest.mark.parametrize("new_mode", [False, True])
def test_applymsg_conflicting_inserts_at_deleted_segment_position(new_mode):
    """client.applyMsg.spec.ts:440-462 (initial state "a----bcd-ef": detached tombstones) -> "ab"."""
    B, c = _clients("a----bcd-ef", new_mode=new_mode)
    seq, ops = 0, []
    seq += 1
    ops.append(c["B"].make(c["B"].local("insert", 4, "B"), seq))
    seq += 1
    ops.append(c["C"].make(c["C"].local("insert", 4, "CC"), seq))
    seq += 1
    ops.append(c["C"].make(c["C"].local("remove", 2, 8), seq))
    c["B"].apply(ops[0])
    c["B"].apply(ops[1])
    seq += 1
    ops.append(c["B"].make(c["B"].local("remove", 5, 8), seq))
    for m in ops:
        for p in c.values():
            if p.current_seq < m["sequenceNumber"]:
                p.apply(m)
    for p in c.values():
        p.check("ab")


def test_applymsg_9703_new_length_calculations():
    """client.applyMsg.spec.ts:464-493 ("Inconsistent shared string after pausing connection #9703",
    mergeTreeUseNewLengthCalculations) -> "ayzXd": the reference's one literal pin of new-length placement."""
    B, c = _clients("abcd", new_mode=True)
    seq, ops = 0, []
    seq += 1
    ops.append(c["B"].make(c["B"].local("remove", 1, 3), seq))
    c["B"].apply(ops[0])
    seq += 1
    ops.append(c["B"].make(c["B"].local("insert", 1, "yz"), seq))
    c["B"].apply(ops[1])
    seq += 1
    ops.append(c["C"].make(c["C"].local("insert", 2, "X"), seq))
    for m in ops:
        for p in c.values():
            if p.current_seq < m["sequenceNumber"]:
                p.apply(m)
    for p in c.values():
        p.check("ayzXd")


class _EngineDump:
    def __init__(self, B, k):
        self.B, self.k = B, k

    def dump_segments(self):
        return self.B.dump_segments(self.k)


@pytest.mark.parametrize("new_mode", [False, True])
def test_inserting_walk_conflict_across_block_boundary_on_the_engine(new_mode):
    """mergeTree.insertingWalk.spec.ts:285-356: seven unacked local inserts at 0 split the root into two
    blocks, "DCBA" removed locally, then a concurrent remote insert at 0 lands directly before "0":
    ["G", "F", "E", "(D)", "(C)", "(B)", "(A)", "x", "0"] (trap T1)."""
    from fluidframework_amd import MergeTreeBatch
    from test_reference_kats import root_child_count, segments
    B = MergeTreeBatch(1, new_length_calc=new_mode)
    c = B[0]
    c.insertTextLocal(0, "0")
    c.startOrUpdateCollaboration("local")
    for i in range(1, 8):
        c.insertTextLocal(0, chr(i + 64))
    B.replay()
    e = _EngineDump(B, 0)
    assert root_child_count(e) == 2
    assert c.getText() == "GFEDCBA0"
    c.removeRangeLocal(3, 7)
    assert c.getText() == "GFE0"
    c.applyMsg(msg("remote", 1, 0, {"type": 0, "pos1": 0, "seg": "x"}))
    B.replay()
    got = [f"({s['text']})" if s["removed"] else s["text"] for s in segments(e)]
    assert got == ["G", "F", "E", "(D)", "(C)", "(B)", "(A)", "x", "0"]


def _zamboni_client():
    """mergeTree.zamboni.spec.ts:15-21: "hello world" inserted locally one character at a time before
    collaboration (detached: 11 segments, the root split 4 / 7), then startOrUpdateCollaboration."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    B = MergeTreeBatch(1)
    c = B[0]
    o = OracleDoc(verify=True)
    for i, ch in enumerate("hello world"):
        c.insertTextLocal(i, ch)
        o.insert_text_local(i, ch)
    c.startOrUpdateCollaboration("localUser")
    o.start_collab("localUser")
    B.replay()
    assert B.dump_segments(0) == o.dump_segments()
    return B, c, o


def _first_block_children(doc):
    from test_reference_kats import segments
    return sum(1 for s in segments(doc) if s["path"][0] == 0)


def test_zamboni_pack_parent_with_no_children_segments_on_the_engine():
    """mergeTree.zamboni.spec.ts:22-43."""
    from test_reference_kats import root_child_count
    B, c, o = _zamboni_client()
    n = c.getLength()
    op = c.removeRangeLocal(0, n - 1)
    assert op == o.remove_local_op(0, n - 1)
    c.applyMsg(msg("localUser", 1, 0, op))
    o.apply_msg(msg("localUser", 1, 0, op))
    c.packParentRoot()
    o.pack_parent_root()
    assert c.getLength() == 1
    cur = o.current_seq
    op = c.removeRangeLocal(0, c.getLength())
    assert op == o.remove_local_op(0, o.get_length())
    m = msg("localUser", cur, cur, op, msn=cur)
    c.applyMsg(m)
    o.apply_msg(m)
    assert c.getLength() == 0
    c.packParentRoot()
    o.pack_parent_root()
    B.replay()
    assert B.dump_segments(0) == o.dump_segments()
    assert root_child_count(_EngineDump(B, 0)) == 0


def test_zamboni_with_no_segments_to_scour_on_the_engine():
    """mergeTree.zamboni.spec.ts:44-52."""
    from test_reference_kats import root_child_count
    B, c, o = _zamboni_client()
    e = _EngineDump(B, 0)
    n, cc = c.getLength(), root_child_count(e)
    c.zamboniSegments()
    B.replay()
    assert (c.getLength(), root_child_count(e)) == (n, cc) == (11, 2)


def test_zamboni_with_one_segment_to_scour_on_the_engine():
    """mergeTree.zamboni.spec.ts:53-66: root.children[0] keeps its child count."""
    B, c, o = _zamboni_client()
    e = _EngineDump(B, 0)
    first, n = _first_block_children(e), c.getLength()
    c.removeRangeLocal(0, 1)
    o.remove_local_op(0, 1)
    c.zamboniSegments()
    o.zamboni()
    B.replay()
    assert c.getLength() == n - 1
    assert _first_block_children(e) == first == 4
    assert B.dump_segments(0) == o.dump_segments()


def test_zamboni_with_many_segments_to_scour_on_the_engine():
    """mergeTree.zamboni.spec.ts:67-79: the first block's length drops to 0 and packParent leaves the root
    one child (the held pending removes plus the coalesced "world")."""
    from test_reference_kats import root_child_count, segments
    B, c, o = _zamboni_client()
    e = _EngineDump(B, 0)
    c.removeRangeLocal(0, 6)
    o.remove_local_op(0, 6)
    B.replay()
    assert all(s["removed"] for s in segments(e) if s["path"][0] == 0)
    c.zamboniSegments()
    c.packParentRoot()
    o.zamboni()
    o.pack_parent_root()
    B.replay()
    assert root_child_count(e) == 1
    assert B.dump_segments(0) == o.dump_segments()
