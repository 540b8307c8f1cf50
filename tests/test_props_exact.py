"""matchProperties where it is no equivalence, and remote "consensus" annotates: the hand-derived known answers
of tests/props_cases.py on the oracle (CPU), and the engine's pack-time handling (the engine's replay parity
is tests/test_gpu_props_exact.py)."""
import json

import pytest

import props_cases as pc
from test_reference_kats import msg


def _run(init, msgs):
    from pyoracle import OracleDoc
    o = OracleDoc(verify=True)
    if init:
        o.insert_text_local(0, init)
    o.start_collab("obs")
    for m in msgs:
        o.apply_msg(m)
    return o


@pytest.mark.parametrize("case", pc.CASES, ids=[c[0] for c in pc.CASES])
def test_known_answers_on_the_oracle(case):
    name, init, msgs, expected = case
    o = _run(init, msgs)
    assert pc.rows(o.dump_segments()) == expected
    # SnapshotV1 coalesces below the MSN with the same head-first comparison (snapshotV1.ts:238-251): here every
    # segment is below the MSN, so the header holds the live rows
    segs = json.loads(o.summarize_v1()["blobs"][0][1])["segments"]
    assert [[s, None] if isinstance(s, str) else [s["text"], s.get("props")] for s in segs] == expected


@pytest.mark.parametrize("case", pc.REFUSED, ids=[c[0] for c in pc.REFUSED])
def test_refused_cases_on_the_oracle(case):
    name, init, msgs, err = case
    with pytest.raises(Exception, match="unsupported"):
        _run(init, msgs)


@pytest.mark.parametrize("case", pc.THROWS, ids=[c[0] for c in pc.THROWS])
def test_reference_failures_on_the_oracle(case):
    name, init, msgs, err = case
    with pytest.raises(Exception, match=err):
        _run(init, msgs)


def test_consensus_values_coalesce_after_a_summary_round_trip():
    """Live, two {value: undefined, seq} values never match (b.value is undefined); loaded from a summary they
    are {"seq": S} objects, which do: the loaded document's own summary coalesces them."""
    from pyoracle import OracleDoc
    o = _run(*pc.CASES[9][1:3])
    blobs = o.summarize_v1()["blobs"]
    p = OracleDoc(verify=True)
    p.load_v1(blobs, "obs2")
    segs = json.loads(p.summarize_v1()["blobs"][0][1])["segments"]
    assert {"text": "cd", "props": {"k": {"seq": 2}}} in segs


def test_consensus_beside_cv_like_values_is_refused_at_apply():
    """A set holding a consensus value matches nothing (like NaN) -- exact as long as its key never holds a
    two-key {value: null | {} | [], seq} object, the one shape matchProperties(cv, y) can accept: that pairing
    is refused, in either order."""
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from test_reference_kats import msg
    cons = {"type": 2, "pos1": 0, "pos2": 1, "props": {"c": 1}, "combiningOp": {"name": "consensus"}}
    like = {"type": 0, "pos1": 0, "seg": {"text": "x", "props": {"c": {"value": None, "seq": 4}}}}
    for first, second in ((like, cons), (cons, like)):
        B = MergeTreeBatch(1)
        B[0].insertTextLocal(0, "abc")
        B[0].startOrUpdateCollaboration("obs")
        B[0].applyMsg(msg("a", 1, 0, first))
        with pytest.raises(MergeTreeError, match=r"\{value, seq\}"):
            B[0].applyMsg(msg("a", 2, 1, second))


def _consensus_marker_log():
    """A live client "me" inserts a marker with id "m1" (acked), annotates it with annotateMarkerNotifyConsensus
    (client.ts:155-181) while remote ops arrive, and receives the ack: the value is {value: undefined, seq: -1}
    (JSON {"seq": -1}) until the ack, then completed in place with the ack's seq (client.ts:1050-1058)."""
    marker = {"type": 0, "pos1": 1, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m1"}}}
    notify = {"type": 2, "props": {"k": 1, "j": 2}, "relativePos1": {"id": "m1", "before": True},
              "relativePos2": {"id": "m1"}, "combiningOp": {"name": "consensus"}, "notifyConsensus": True}
    return marker, notify


def test_local_consensus_through_annotate_marker_notify_consensus():
    from pyoracle import OracleDoc
    marker, notify = _consensus_marker_log()
    o = OracleDoc(verify=True)
    o.insert_text_local(0, "abcd")
    o.start_collab("me")
    sent_marker = o.local_op_json(marker)
    o.apply_msg(msg("me", 1, 0, sent_marker))
    o.apply_msg(msg("x", 2, 1, {"type": 2, "pos1": 0, "pos2": 5, "props": {"j": 7}}))
    sent = o.local_op_json(notify)
    assert "notifyConsensus" not in sent and sent["relativePos1"] == {"id": "m1", "before": True}
    rows = [r[7] for r in json.loads("[" + ",".join(o.dump_segments().splitlines()[1:]) + "]") if r[1] == "M"]
    assert rows == [{"markerId": "m1", "j": 7, "k": {"seq": -1}}], rows  # (j stays: a present value stays)
    o.apply_msg(msg("x", 3, 2, {"type": 0, "pos1": 0, "seg": "Z"}))
    o.apply_msg(msg("me", 4, 2, sent, msn=2))
    rows = [r[7] for r in json.loads("[" + ",".join(o.dump_segments().splitlines()[1:]) + "]") if r[1] == "M"]
    assert rows == [{"markerId": "m1", "j": 7, "k": {"seq": 4}}], rows


def test_plain_local_consensus_is_refused():
    from pyoracle import OracleDoc
    marker, notify = _consensus_marker_log()
    o = OracleDoc()
    o.insert_text_local(0, "abcd")
    o.start_collab("me")
    o.apply_msg(msg("me", 1, 0, o.local_op_json(marker)))
    del notify["notifyConsensus"]
    with pytest.raises(Exception, match="annotateMarkerNotifyConsensus"):
        o.local_op_json(notify)
