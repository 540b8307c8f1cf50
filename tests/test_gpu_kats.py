"""The all-remote reference KATs of tests/test_reference_kats.py on the GPU engine (an observer sees every
op as a sequenced remote message): expected texts / lengths from the reference tests, and the canonical
segment dump equal to the oracle replaying the same messages.

* mergeTree.markRangeRemoved.spec.ts:114-154 and the passive observer of :156-227;
* partialLength.spec.ts:39-297, the remote-client tables (a view's length is the sum of mapRange over it);
* mergeTree.annotate.spec.ts:529-575 (a remote annotate; a later split copies its properties).
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
