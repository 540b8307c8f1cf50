"""GPU parity of matchProperties where it is no equivalence (properties.ts:71-96: primitive against object,
string against index object, nested nulls, consensus values) and of remote "consensus" annotates
(properties.ts:46-62); the engine tabulates such keys pair by pair (mtb_host.cpp Interner::irr_tables) and
compares each segment with its run's head in zamboni and SnapshotV1.

Bar: bit-exact against the oracle (canonical dump, text, state digest, SnapshotV1 blobs) on
* the hand-derived known answers of tests/props_cases.py (CPU: tests/test_props_exact.py), rows included;
* generated logs (helpers.make_props_log), both length modes, two flushes, then a SnapshotV1 round trip
  loaded by the engine and continued;
* the refused case (an object value whose seq is -1) and the reference's own failure (a null consensus
  defaultValue: a TypeError there, MTB_E_ASSERT here): the engine fails that document
  loudly (DERR_CONSENSUS), the other documents of the batch replay."""
import pytest

import props_cases as pc
from helpers import first_diff, make_props_log

pytestmark = pytest.mark.gpu


def _same(B, i, o, what):
    gd, od = B.dump_segments(i), o.dump_segments()
    assert gd == od, f"{what}: segment dump differs: {first_diff(gd, od)}"
    assert B.text(i) == o.get_text(), f"{what}: text differs"
    assert B.digests(i, 1)[0] == o.digest(), f"{what}: digest differs"
    gb, gs = B.summarize_v1(i)
    assert [list(x) for x in gb] == o.summarize_v1()["blobs"], f"{what}: SnapshotV1 differs"


def test_known_answers_on_the_engine():
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    B = MergeTreeBatch(len(pc.CASES))
    orc = []
    for i, (name, init, msgs, _) in enumerate(pc.CASES):
        o = OracleDoc()
        if init:
            B[i].insertTextLocal(0, init)
            o.insert_text_local(0, init)
        B[i].startOrUpdateCollaboration("obs")
        o.start_collab("obs")
        for m in msgs:
            B[i].applyMsg(m)
            o.apply_msg(m)
        orc.append(o)
    st = B.flush()
    assert st["errors"] == 0, st
    for i, (name, _, _, expected) in enumerate(pc.CASES):
        assert pc.rows(B.dump_segments(i)) == expected, name
        _same(B, i, orc[i], name)


def test_refused_cases_fail_their_documents_only():
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from pyoracle import OracleDoc
    good = pc.CASES[9]
    docs = [c[1:3] for c in pc.REFUSED + pc.THROWS] + [good[1:3]]
    B = MergeTreeBatch(len(docs))
    for i, (init, msgs) in enumerate(docs):
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("obs")
        for m in msgs:
            B[i].applyMsg(m)
    with pytest.raises(MergeTreeError, match="consensus"):
        B.flush()
    for c in pc.REFUSED + pc.THROWS:  # each alone: its own error (THROWS: the reference's own failure, MTB_E_ASSERT)
        one = MergeTreeBatch(1)
        one[0].insertTextLocal(0, c[1])
        one[0].startOrUpdateCollaboration("obs")
        for m in c[2]:
            one[0].applyMsg(m)
        with pytest.raises(MergeTreeError, match=c[3] if c in pc.THROWS else "unsupported") as ei:
            one.flush()
        assert ei.value.code == (-4 if c in pc.THROWS else -6), (c[0], ei.value.code)
    o = OracleDoc()
    o.insert_text_local(0, good[1])
    o.start_collab("obs")
    for m in good[2]:
        o.apply_msg(m)
    _same(B, len(docs) - 1, o, "good document")


@pytest.mark.parametrize("new_mode", [False, True])
def test_property_logs(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    logs = [make_props_log(700 + s + 20 * int(new_mode), 1200, n_clients=3 + s % 4, lag=4 + 6 * s, new_mode=new_mode)
            for s in range(10)]
    B = MergeTreeBatch(len(logs), new_length_calc=new_mode)
    orc = []
    for i, (init, _) in enumerate(logs):
        B[i].insertTextLocal(0, init)
        B[i].startOrUpdateCollaboration("obs")
        o = OracleDoc(new_length_calc=new_mode)
        o.insert_text_local(0, init)
        o.start_collab("obs")
        orc.append(o)
    for part in (slice(0, 600), slice(600, None)):
        for i, (_, msgs) in enumerate(logs):
            for m in msgs[part]:
                B[i].applyMsg(m)
                orc[i].apply_msg(m)
        st = B.replay()
        assert st["errors"] == 0, st
        for i, o in enumerate(orc):
            _same(B, i, o, f"log {i} {part}")


@pytest.mark.parametrize("new_mode", [False, True])
def test_property_logs_through_a_summary(new_mode):
    """Summarize mid-log (values outside any equivalence, consensus values as {"seq": S}), load the summary on
    the engine and the oracle, continue both with the rest of the log."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    logs = [make_props_log(900 + s + 20 * int(new_mode), 800, n_clients=3, lag=6, new_mode=new_mode)
            for s in range(6)]
    B = MergeTreeBatch(len(logs), new_length_calc=new_mode)
    orc = []
    for i, (init, msgs) in enumerate(logs):
        g = OracleDoc(new_length_calc=new_mode)
        g.insert_text_local(0, init)
        g.start_collab("obs")
        for m in msgs[:500]:
            g.apply_msg(m)
        blobs = g.summarize_v1()["blobs"]
        B[i].load(blobs, "loader")
        o = OracleDoc(new_length_calc=new_mode)
        o.load_v1(blobs, "loader")
        for m in msgs[500:]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        orc.append(o)
    st = B.flush()
    assert st["errors"] == 0, st
    for i, o in enumerate(orc):
        _same(B, i, o, f"log {i}")


def test_many_consensus_values_in_one_batch():
    """Every remote consensus annotate makes a new value per key ({value: undefined, seq}); a batch of many
    documents holds thousands under one key.  They never make the key irregular (their sets match nothing,
    MTB_PNAN), so no pair table grows with them."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    from test_reference_kats import msg
    import random
    n = 24
    B = MergeTreeBatch(n)
    orc = []
    for i in range(n):
        rng = random.Random(900 + i)
        o = OracleDoc()
        B[i].insertTextLocal(0, "consensus " * 8)
        o.insert_text_local(0, "consensus " * 8)
        B[i].startOrUpdateCollaboration("obs")
        o.start_collab("obs")
        length = 80
        for s in range(1, 301):
            a = rng.randrange(length - 1)
            if rng.random() < 0.7:
                op = {"type": 2, "pos1": a, "pos2": min(length, a + rng.randint(1, 6)), "props": {"c": 1},
                      "combiningOp": {"name": "consensus"}}
            elif rng.random() < 0.5:
                op = {"type": 0, "pos1": a, "seg": rng.choice(["ab", "c"])}
                length += len(op["seg"])
            else:
                op = {"type": 2, "pos1": a, "pos2": a + 1, "props": {"c": rng.choice([1, None, "z"])}}
            m = msg(f"client-{s % 3}", s, s - 1 - rng.randint(0, 3) if s > 4 else s - 1, op, msn=max(0, s - 6))
            B[i].applyMsg(m)
            o.apply_msg(m)
        orc.append(o)
    st = B.flush()
    assert st["errors"] == 0, st
    for i, o in enumerate(orc):
        _same(B, i, o, f"doc {i}")
