"""A live client's own consensus annotates: Client.annotateMarkerNotifyConsensus (client.ts:155-181) gives each key
{value: undefined, seq: -1} on the marker until the op's ack, where updateConsensusProperty (:1050-1058) completes
the marker's value with the ack's seq (tests/test_props_exact.py pins the oracle by hand).  Bar: the engine's
canonical dump, text, digest and SnapshotV1 equal the oracle's after every replay, on the known answer and on a
randomized farm of remote edits, remote consensus on other keys, and notify-consensus annotates acked with lag."""
import json
import random

import pytest

from helpers import first_diff
from test_reference_kats import msg

pytestmark = pytest.mark.gpu


def _pair(initial="abcd"):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    B = MergeTreeBatch(1)
    B[0].insertTextLocal(0, initial)
    B[0].startOrUpdateCollaboration("me")
    o = OracleDoc(verify=True)
    o.insert_text_local(0, initial)
    o.start_collab("me")
    return B, o


def _same(B, o, what):
    B.replay()
    gd, od = B.dump_segments(0), o.dump_segments()
    assert gd == od, f"{what}: segment dump differs: {first_diff(gd, od)}"
    assert B.text(0) == o.get_text()
    assert B.digests(0, 1)[0] == o.digest(), what


def test_notify_consensus_known_answer():
    B, o = _pair()
    marker = {"type": 0, "pos1": 1, "seg": {"marker": {"refType": 1}, "props": {"markerId": "m1"}}}
    B[0].applyLocalOp(marker)
    o.local_op_json(marker)
    for m in (msg("me", 1, 0, marker), msg("x", 2, 1, {"type": 2, "pos1": 0, "pos2": 5, "props": {"j": 7}})):
        B[0].applyMsg(m)
        o.apply_msg(m)
    sent = B[0].annotateMarkerNotifyConsensus("m1", {"k": 1, "j": 2})
    assert sent == o.local_op_json(dict(sent, notifyConsensus=True))
    _same(B, o, "pending")
    assert '"k":{"seq":-1}' in B.dump_segments(0)
    for m in (msg("x", 3, 2, {"type": 0, "pos1": 0, "seg": "Z"}), msg("me", 4, 2, sent, msn=2)):
        B[0].applyMsg(m)
        o.apply_msg(m)
    _same(B, o, "acked")
    assert '"k":{"seq":4}' in B.dump_segments(0) and '"j":7' in B.dump_segments(0)
    gb, _ = B.summarize_v1(0)
    assert [list(x) for x in gb] == o.summarize_v1()["blobs"]


@pytest.mark.parametrize("seed", range(4))
def test_notify_consensus_farm(seed):
    rng = random.Random(seed)
    B, o = _pair("hello consensus world")
    ids = ["m0", "m1", "m2"]
    seq = 0
    for k, mid in enumerate(ids):  # the markers, inserted and acked first
        op = {"type": 0, "pos1": 3 + 5 * k, "seg": {"marker": {"refType": 1}, "props": {"markerId": mid}}}
        B[0].applyLocalOp(op)
        o.local_op_json(op)
        seq += 1
        m = msg("me", seq, seq - 1, op, msn=seq - 1)
        B[0].applyMsg(m)
        o.apply_msg(m)
    pending = []  # (op, refSeq when sent)
    msn = seq
    for step in range(80):
        r = rng.random()
        if 0.35 <= r < 0.7:
            mid = rng.choice(ids)
            props = rng.choice([{"k": 1}, {"k": 1, "q": 2}, {"j": 5}])
            sent = B[0].annotateMarkerNotifyConsensus(mid, props)
            assert sent == o.local_op_json(dict(sent, notifyConsensus=True))
            pending.append((sent, seq))
            continue
        if r < 0.35 or not pending:
            n = o.get_length()
            x = rng.random()
            if x < 0.4:
                contents = {"type": 0, "pos1": rng.randint(0, n), "seg": rng.choice(["ab", "c", "xyz"])}
            elif x < 0.6 and n > 4:
                p1 = rng.randrange(n - 1)
                contents = {"type": 1, "pos1": p1, "pos2": min(n, p1 + rng.randint(1, 2))}
            else:
                p1 = rng.randrange(n)
                comb = {"name": "consensus"} if rng.random() < 0.3 else None
                # (remote consensus names a key this client never consensus-annotates: over a pending {seq: -1}
                # object it would complete that object in place -- refused on both sides)
                contents = {"type": 2, "pos1": p1, "pos2": min(n, p1 + rng.randint(1, 6)),
                            "props": {"z" if comb else rng.choice(["j", "q"]): rng.randint(0, 3)}}
                if comb:
                    contents["combiningOp"] = comb
            seq += 1
            m = msg(rng.choice(["x", "y"]), seq, seq - 1, contents, msn=msn)
        else:
            sent, ref = pending.pop(0)
            seq += 1
            m = msg("me", seq, ref, sent, msn=msn)
        msn = min([seq] + [ref for _, ref in pending])
        m["minimumSequenceNumber"] = min(m["minimumSequenceNumber"], msn)
        B[0].applyMsg(m)
        o.apply_msg(m)
        if step % 7 == 6:
            _same(B, o, f"seed {seed} step {step}")
    _same(B, o, f"seed {seed} end")
    gb, _ = B.summarize_v1(0)
    assert [list(x) for x in gb] == o.summarize_v1()["blobs"]
