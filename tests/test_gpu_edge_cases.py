"""GPU parity on edge cases in one ragged batch (the shapes the reference's own tests exercise).

One MergeTreeBatch holds documents of very different kinds and lengths, replayed by the same launches:
an empty document, long inserts (> 256 units, split and never appended by zamboni), markers with
props, annotates with many keys (null deletes, nested values, key order), GROUP ops, removal of the
whole document followed by inserts, newline / surrogate-pair text (TextSegment.canAppend), a single
writer at lag 0 (zamboni coalescing), 8 writers at lag 128, and a document that fails in the kernel
("MergeTree insert failed") while its neighbours continue.  Bar: bit-exact vs the oracle — text, the
canonical segment dump and the SnapshotV1 blobs; the failing document's error is raised once, by the
flush that hit it, and its state stays the one before the failing op.
Every message is generated valid in its author's (refSeq, client) view by driving the oracle.
"""
import random

import pytest

from helpers import first_diff

pytestmark = pytest.mark.gpu

TEXTS = ["abc", "\n", "x\ny", "\U0001F600", "éè", "z" * 300, "q" * 5000]
PROPS = [{"bold": True}, {"bold": None}, {"color": "red", "size": 12, "font": {"face": "x", "w": 2}},
         {"1": 4, "b": 1, "a": 3, "2": 2}, {"a": None, "b": None, "k": [1, 2, {"z": 3}]}, {"size": 12.5}]


def _gen(seed, n_msgs, n_clients, lag, kinds, new_mode):
    """Messages for one document, generated against an oracle observer."""
    from pyoracle import OracleDoc
    rng = random.Random(seed)
    o = OracleDoc(new_length_calc=new_mode)
    o.insert_text_local(0, "seed text\nwith a newline")
    o.start_collab("obs")
    clients = [f"c{k}" for k in range(n_clients)]
    ref = {c: 0 for c in clients}
    msgs, seq = [], 0
    for _ in range(n_msgs):
        w = rng.choice(clients)
        ref[w] = max(ref[w], seq - rng.randint(0, lag))
        r = ref[w]
        o.add_client(w)
        ln = o.remote_length(r, o.client_ids().index(w))
        seq += 1

        def u16(t):
            return len(t.encode("utf-16-le")) // 2

        def one(ln):
            k = rng.choice(kinds)
            if k == "marker" and ln >= 0:
                seg = {"marker": {"refType": rng.choice([0, 1, 2])}}
                if rng.random() < 0.5:
                    seg["props"] = {"markerId": f"m{seq}", "tile": True}
                return {"type": 0, "pos1": rng.randint(0, ln), "seg": seg}, 1
            if k in ("insert", "group") or ln == 0:
                t = rng.choice(TEXTS)
                seg = {"text": t, "props": rng.choice(PROPS[:1] + PROPS[2:4])} if rng.random() < 0.2 else t
                return {"type": 0, "pos1": rng.randint(0, ln), "seg": seg}, u16(t)
            a = rng.randrange(ln)
            b = min(ln, a + rng.randint(1, 40))
            if k == "remove_all":
                a, b = 0, ln
            if k in ("remove", "remove_all"):
                return {"type": 1, "pos1": a, "pos2": b}, -(b - a)
            return {"type": 2, "pos1": a, "pos2": b, "props": rng.choice(PROPS)}, 0

        if "group" in kinds and rng.random() < 0.25:
            ops = []
            for _ in range(rng.randint(1, 3)):
                op, dl = one(ln)
                ops.append(op)
                ln += dl  # members see the earlier members of the same client's group
            contents = {"type": 3, "ops": ops}
        else:
            contents, _ = one(ln)
        msg = {"clientId": w, "sequenceNumber": seq, "referenceSequenceNumber": r,
               "minimumSequenceNumber": min(ref.values()), "type": "op", "contents": contents}
        o.apply_msg(msg)
        msgs.append(msg)
    return msgs


def _docs(new_mode):
    base = ["insert", "insert", "remove", "annotate"]
    return [
        [],                                                                       # empty document
        _gen(1, 300, 1, 0, base, new_mode),                                       # one writer, lag 0
        _gen(2, 600, 8, 128, base + ["marker"], new_mode),                        # 8 writers, lag 128
        _gen(3, 400, 4, 20, base + ["group", "marker"], new_mode),                # GROUP ops
        _gen(4, 200, 3, 10, ["insert", "remove_all", "insert", "annotate"], new_mode),  # whole-doc removes
        _gen(5, 300, 5, 40, ["annotate", "annotate", "insert", "remove"], new_mode),   # many-key annotates
        _gen(6, 3000, 6, 64, base, new_mode),                                     # long document
    ]


@pytest.mark.parametrize("new_mode", [False, True])
def test_ragged_batch_edge_cases_match_oracle(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.client import MergeTreeError
    from pyoracle import OracleDoc
    docs = _docs(new_mode)
    B = MergeTreeBatch(len(docs) + 1, new_length_calc=new_mode, chunk_size=500)
    oracles = []
    for i, msgs in enumerate(docs):
        B[i].insertTextLocal(0, "seed text\nwith a newline")
        B[i].startOrUpdateCollaboration("obs")
        o = OracleDoc(new_length_calc=new_mode, chunk_size=500)
        o.insert_text_local(0, "seed text\nwith a newline")
        o.start_collab("obs")
        half = len(msgs) // 3
        for m in msgs[:half]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append((o, msgs[half:]))
    # the failing document: a remote insert past the end ("MergeTree insert failed", mergeTree.ts:1671),
    # found by the kernel; an out-of-order sequence number (assert 0x038, client.ts:880) throws at apply
    bad = len(docs)
    B[bad].startOrUpdateCollaboration("obs")
    B[bad].applyMsg({"clientId": "w", "sequenceNumber": 5, "referenceSequenceNumber": 0, "minimumSequenceNumber": 0,
                     "type": "op", "contents": {"type": 0, "pos1": 0, "seg": "ok"}})
    with pytest.raises(MergeTreeError, match="0x038"):
        B[bad].applyMsg({"clientId": "w", "sequenceNumber": 3, "referenceSequenceNumber": 0,
                         "minimumSequenceNumber": 0, "type": "op", "contents": {"type": 0, "pos1": 0, "seg": "no"}})
    B[bad].applyMsg({"clientId": "w", "sequenceNumber": 6, "referenceSequenceNumber": 5, "minimumSequenceNumber": 0,
                     "type": "op", "contents": {"type": 0, "pos1": 50, "seg": "past the end"}})
    # an unknown combiningOp is outside the engine's subset: rejected loudly at apply
    with pytest.raises(MergeTreeError, match="unsupported"):
        B[1].applyMsg({"clientId": "c0", "sequenceNumber": 10 ** 6, "referenceSequenceNumber": 0,
                       "minimumSequenceNumber": 0, "type": "op",
                       "contents": {"type": 2, "pos1": 0, "pos2": 1, "props": {"k": 1}, "combiningOp": {"name": "max"}}})
    # first third, then the rest: both flushes replay the whole ragged batch.  The failure is reported
    # once, by the flush whose replay hit it; the other documents' records were replayed by it.
    with pytest.raises(MergeTreeError, match=r"document 7 op \d+: MergeTree insert failed"):
        B.flush()
    for i, (o, rest) in enumerate(oracles):
        for m in rest:
            B[i].applyMsg(m)
            o.apply_msg(m)
    st = B.flush()
    assert st["errors"] == 1
    for i, (o, _) in enumerate(oracles):
        assert B.text(i) == o.get_text(), f"doc {i}: text"
        gd, od = B.dump_segments(i), o.dump_segments()
        assert gd == od, f"doc {i}: dump differs: {first_diff(gd, od)}"
        gb, gs = B.summarize_v1(i)
        osum = o.summarize_v1()
        assert [list(x) for x in gb] == osum["blobs"], f"doc {i}: summary blobs"
        assert gs == osum["summary"], f"doc {i}: summary tree"
    assert B.text(bad) == "ok"  # the state before the failing op (blockInsert throws before mutating)


@pytest.mark.parametrize("new_mode", [False, True])
def test_segment_queries_match_oracle(new_mode):
    """Client.getContainingSegment (local view and remote perspectives), getPropertiesAtPosition and
    walkSegments (client.ts:286, 1065, 1101) read the engine's state; the oracle answers the same queries
    through its own nodeMap over partial lengths (mergeTree.ts:2531)."""
    import random as _r
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    msgs = _gen(21, 800, 6, 96, ["insert", "insert", "remove", "annotate", "marker"], new_mode)
    B = MergeTreeBatch(1, new_length_calc=new_mode)
    B[0].insertTextLocal(0, "seed text\nwith a newline")
    B[0].startOrUpdateCollaboration("obs")
    o = OracleDoc(new_length_calc=new_mode)
    o.insert_text_local(0, "seed text\nwith a newline")
    o.start_collab("obs")
    rng = _r.Random(5)
    for k, m in enumerate(msgs):
        B[0].applyMsg(m)
        o.apply_msg(m)
        if k % 200 != 199:
            continue
        assert B.map_range(0) == o.map_range(), f"walk after {k + 1}"
        n = o.get_length()
        for pos in rng.sample(range(n), min(n, 40)):
            assert B.map_range(0, pos, pos + 1, limit=1) == o.map_range(pos, pos + 1, limit=1), f"pos {pos}"
            seg = B[0].getContainingSegment(pos)
            assert seg["segment"] is not None and 0 <= seg["offset"] < seg["segment"]["cachedLength"]
        # remote perspectives: each client at a lagging refSeq inside the collab window (a sequenced op's
        # refSeq is never below the MSN; below it the partial lengths have folded the history away)
        cur, msn = o.current_seq, o.min_seq
        for cid in ["c0", "c1", "c5", "never-seen"]:
            ref = rng.randint(msn, cur)
            assert B.map_range(0, 0, -1, ref, cid) == o.map_range(0, -1, ref, cid), f"{cid}@{ref}"
            rl = len(o.map_range(0, -1, ref, cid))
            if rl:
                assert B.map_range(0, 3, 40, ref, cid) == o.map_range(3, 40, ref, cid)
    props = [B[0].getPropertiesAtPosition(p) for p in range(0, o.get_length(), 7)]
    assert props == [(o.map_range(p, p + 1, limit=1)[0]["segment"].get("properties")) for p in range(0, o.get_length(), 7)]
    seen = []
    B[0].walkSegments(lambda s, pos, *_: seen.append((pos, s["cachedLength"])) or len(seen) < 50, 5, 400)
    assert seen == [(e["pos"], e["segment"]["cachedLength"]) for e in o.map_range(5, 400)][:50]
