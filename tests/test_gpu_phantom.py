"""GPU parity of SnapshotV1 loads whose body holds removed segments inserted by collaborating clients: the
reference's phantom partial lengths (tests/phantom_cases.py; mtb_replay.hip "phantom partial lengths").
Bar: the engine equals the oracle -- dump, text, summary -- after the load and after later remote ops:
* the hand-derived known answer (text "h1234567ZY", not the exact-lengths "h1234567YZ");
* constructed summaries with client-inserted segments, removed or not, in header and body chunks;
* synthetic documents of more than 10,000 characters summarized mid-collaboration (SnapshotV1's default
  chunk size, so the removed collaborator-inserted segments past char 10,000 are body segments) and a small
  chunk size, loaded, then the rest of each log replayed."""
import json

import pytest

import phantom_cases as pc
from helpers import first_diff, make_v1_summary, records_to_msgs

pytestmark = pytest.mark.gpu


def _same(B, i, o, what):
    gd, od = B.dump_segments(i), o.dump_segments()
    assert gd == od, f"{what}: segment dump differs: {first_diff(gd, od)}"
    assert B.text(i) == o.get_text(), f"{what}: text differs"
    gb, gs = B.summarize_v1(i)
    assert [list(x) for x in gb] == o.summarize_v1()["blobs"], f"{what}: SnapshotV1 blobs differ"


def _phantoms(blobs):
    n = 0
    for path, content in blobs[1:]:
        for s in json.loads(content)["segments"]:
            n += isinstance(s, dict) and "client" in s and "removedSeq" in s
    return n


@pytest.mark.parametrize("new_mode", [False, True])
def test_phantom_kat_on_the_engine(new_mode):
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode)
    o.load_v1(pc.kat_summary(), "L")
    B = MergeTreeBatch(1, new_length_calc=new_mode)
    B[0].load(pc.kat_summary(), "L")
    B.flush()
    _same(B, 0, o, "after load")
    # Client.getContainingSegment / walkSegments in remote views: the reference's nodeMap walks block partial
    # lengths, so positions past L2 move by the surplus where pp's removal is visible
    for ref, cid in ((15, "c"), (12, "a"), (11, "d"), (20, "b"), (-1, None)):
        assert B.map_range(0, 0, -1, ref, cid) == o.map_range(0, -1, ref, cid), f"{cid}@{ref}"
        for pos in range(0, 14):
            assert B.map_range(0, pos, pos + 1, ref, cid, limit=1) == o.map_range(pos, pos + 1, ref, cid, limit=1)
    for m in pc.kat_msgs():
        B[0].applyMsg(m)
        o.apply_msg(m)
    B.flush()
    assert B.text(0) == pc.KAT_TEXT
    _same(B, 0, o, "after the two inserts")


@pytest.mark.parametrize("new_mode", [False, True])
def test_deficit_kat_on_the_engine(new_mode):
    """addSeq over an existing entry below newer ones (tests/phantom_cases.py def_summary): the client term shorts
    a's view below t1c, the main term c's view from t1 on -- "h1234567ABCDEFZY", not "h1234567ABCDEZYF"."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode)
    o.load_v1(pc.def_summary(), "L")
    assert o.stale_deficits() == 1
    B = MergeTreeBatch(1, new_length_calc=new_mode)
    B[0].load(pc.def_summary(), "L")
    B.flush()
    _same(B, 0, o, "after load")
    # nodeMap in remote views walks the same partial lengths: positions past L2 move by the deficit
    for ref, cid in ((12, "a"), (14, "a"), (15, "a"), (16, "c"), (12, "c"), (20, "b"), (-1, None)):
        assert B.map_range(0, 0, -1, ref, cid) == o.map_range(0, -1, ref, cid), f"{cid}@{ref}"
        for pos in range(0, 18):
            assert B.map_range(0, pos, pos + 1, ref, cid, limit=1) == o.map_range(pos, pos + 1, ref, cid, limit=1)
    for m in pc.def_msgs():
        B[0].applyMsg(m)
        o.apply_msg(m)
    B.flush()
    assert B.text(0) == pc.DEF_TEXT
    _same(B, 0, o, "after the two inserts")


def _tail_summary(seed, n_noncollab, n_client, chunk_len, msn=10, seq=40):
    """A constructed SnapshotV1 summary the reference can load: NonCollab segments first (some removed above
    the MSN by 1-3 clients), then segments of one inserting client above the MSN, a third of them removed by
    any clients (body segments of several inserting clients, or NonCollab ones after client ones, fall outside
    the (refSeq 0, client) view the loader appends them in: "MergeTree insert failed").  As in any summary a
    collaboration writes, each seq above the MSN is one op of one client: an insert of the inserting client, or
    a remove whose client is the first of removedClientIds (the others removed the same segment later)."""
    import random
    rng = random.Random(seed)
    clients = [f"client-{k}" for k in range(4)]
    ins = clients[seed % 4]
    owner = {q: rng.choice(clients) for q in range(msn + 1, seq + 1)}
    ins_seqs = [q for q in range(msn + 1, seq) if owner[q] == ins and rng.random() < 0.7] or [msn + 1]
    rem_seqs = [q for q in range(msn + 1, seq + 1) if q not in ins_seqs]

    def removers(r, most):
        others = [c for c in clients if c != owner[r]]
        return [owner[r]] + rng.sample(others, rng.randint(0, most))
    segs = []
    for i in range(n_noncollab + n_client):
        t = "".join(rng.choice("abcdefgh \n") for _ in range(rng.randint(1, 9)))
        spec = t if rng.random() < 0.7 else {"text": t, "props": {"bold": True}}
        if i < n_noncollab:
            if rng.random() < 0.2:
                r = rng.choice(rem_seqs)
                spec = {"json": spec, "removedSeq": r, "removedClientIds": removers(r, 2)}
        else:
            sq = rng.choice(ins_seqs)
            spec = {"json": spec, "client": ins, "seq": sq}
            later = [q for q in rem_seqs if q > sq]
            if later and rng.random() < 0.35:
                r = rng.choice(later)
                spec["removedSeq"] = r
                spec["removedClientIds"] = removers(r, 1)
        segs.append((spec, len(t)))
    chunks, cur, cur_len = [], [], 0
    for spec, ln in segs:
        cur.append(spec)
        cur_len += ln
        if cur_len >= chunk_len:
            chunks.append(cur)
            cur, cur_len = [], 0
    if cur:
        chunks.append(cur)
    ids = ["header"] + [f"body_{k}" for k in range(len(chunks) - 1)]
    blobs, start = [], 0
    for k, c in enumerate(chunks):
        o = {"version": "1", "segmentCount": len(c), "length": 0, "segments": c, "startIndex": start}
        if k == 0:
            o["headerMetadata"] = {"minSequenceNumber": msn, "sequenceNumber": seq,
                                   "orderedChunkMetadata": [{"id": x} for x in ids],
                                   "totalLength": 0, "totalSegmentCount": len(segs)}
        start += len(c)
        blobs.append([ids[k], json.dumps(o, separators=(",", ":"))])
    return blobs


def _load_and_continue(blobs, tail, new_mode, chunk=0):
    """Load `blobs` on the oracle and on the engine, then apply `tail`.  The reference's outcome decides:
    * "MergeTree insert failed" at load or at a later op -- the engine fails the same step;
    * otherwise the engine's state equals the oracle's after the load and after the tail, also where a body
      insert's incremental update replaced the seglen of an existing entry below newer ones (the oracle counts
      these, stale_deficits: addSeq leaves the later cumulative lengths short; the engine's deficit table).
    Returns "failed", "equal" or "deficit" (equal, with deficits)."""
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from pyoracle import OracleDoc
    o = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
    B = MergeTreeBatch(1, new_length_calc=new_mode, chunk_size=chunk)
    B[0].load(blobs, "loader")
    try:
        o.load_v1(blobs, "loader")
        o.get_text()
        ofail = None
    except Exception as e:
        assert "MergeTree insert failed" in str(e), str(e)
        ofail = str(e)
    try:
        B.flush()
    except MergeTreeError as e:
        assert ofail is not None and "MergeTree insert failed" in str(e), str(e)
        return "failed"
    assert ofail is None, "the engine loaded a summary the reference cannot"
    _same(B, 0, o, "after load")
    for m in tail:
        try:
            o.apply_msg(m)
        except Exception as e:
            assert "MergeTree insert failed" in str(e)
            B[0].applyMsg(m)
            with pytest.raises(MergeTreeError, match="MergeTree insert failed"):
                B.flush()
            return "failed"
        B[0].applyMsg(m)
    B.flush()
    _same(B, 0, o, "after load + tail")
    return "deficit" if o.stale_deficits() else "equal"


@pytest.mark.parametrize("new_mode", [False, True])
def test_constructed_summaries_with_removed_client_segments_in_the_body(new_mode):
    from pyoracle import OracleDoc
    from test_gpu_load import _remote_tail
    out = []
    for i in range(24):
        blobs = _tail_summary(500 + i, 120 + 20 * i, 60 + 5 * i, 100 + 10 * (i % 5))
        g = OracleDoc(new_length_calc=new_mode)
        try:
            g.load_v1(blobs, "obs")
            tail = _remote_tail(g, 11 * i, 150, 40, 10, ["client-0", "client-1", "client-7"])
        except Exception:
            tail = []
        out.append(_load_and_continue(blobs, tail, new_mode))
    assert set(out) <= {"deficit", "failed", "equal"} and "deficit" in out


def _rising_tail(o, seed, n_ops, start_seq, msn_lag=3, out=None):
    """Remote ops after a load whose MSN trails the seq by `msn_lag` (each author has seen everything): blocks the
    ops update copy their deficits down into minLength (partialLengths.ts:809-819), and recombinations then carry
    them up (:304-308) -- or drop the ones not copied down yet."""
    import random
    rng = random.Random(seed)
    msgs = [] if out is None else out
    seq = start_seq
    for _ in range(n_ops):
        seq += 1
        ln = o.get_length()
        r = rng.random()
        if ln == 0 or r < 0.5:
            contents = {"type": 0, "pos1": rng.randint(0, ln), "seg": "".join(rng.choice("xyz\n") for _ in range(rng.randint(1, 6)))}
        else:
            p1 = rng.randint(0, ln - 1)
            p2 = min(ln, p1 + rng.randint(1, 8))
            contents = {"type": 1, "pos1": p1, "pos2": p2} if r < 0.8 else \
                {"type": 2, "pos1": p1, "pos2": p2, "props": {"bold": rng.choice([True, None])}}
        m = {"clientId": rng.choice(["client-0", "client-1", "client-7"]), "sequenceNumber": seq,
             "referenceSequenceNumber": seq - 1, "minimumSequenceNumber": max(10, seq - msn_lag), "type": "op",
             "contents": contents}
        msgs.append(m)
        o.apply_msg(m)  # (raises at an op the reference fails: msgs ends with it)
    return msgs


@pytest.mark.parametrize("new_mode", [False, True])
def test_small_summaries_with_deficits(new_mode):
    """Small constructed summaries (4-16 NonCollab, 3-19 client segments, chunks of 6-12 chars) whose loads leave
    deficits in the reference, in one batch: the engine equals the oracle after the load and after 60 remote ops
    with a rising MSN (or 30 with the MSN held at 10); where the reference fails one of the 60 ("MergeTree insert
    failed": the deficits put its position past the blocks' lengths), the engine fails that op too."""
    from fluidframework_amd import MergeTreeBatch, MergeTreeError
    from pyoracle import OracleDoc
    from test_gpu_load import _remote_tail
    cases, fails = [], []
    for k in range(300):
        blobs = _tail_summary(7000 + k, 4 + k % 13, 3 + (k // 13) % 17, 6 + k % 7)
        o = OracleDoc(new_length_calc=new_mode)
        try:
            o.load_v1(blobs, "loader")
        except Exception:
            continue
        if not o.stale_deficits():
            continue
        g = OracleDoc(new_length_calc=new_mode)
        g.load_v1(blobs, "obs")
        if k % 2:
            try:
                tail = _remote_tail(g, k, 30, 40, 10, ["client-0", "client-1", "client-7"])
            except Exception:
                continue
        else:
            tail = []
            try:
                tail = _rising_tail(g, k, 60, 40, out=tail)
            except Exception as e:  # the reference fails a later insert: the engine must fail the same op
                assert "MergeTree insert failed" in str(e)
                fails.append((blobs, tail))
                continue
        cases.append((blobs, o, tail))
    assert len(cases) >= 100
    B = MergeTreeBatch(len(cases), new_length_calc=new_mode)
    for j, (blobs, o, tail) in enumerate(cases):
        B[j].load(blobs, "loader")
    B.flush()
    for j, (blobs, o, tail) in enumerate(cases):
        _same(B, j, o, f"case {j} after load")
        for m in tail:
            B[j].applyMsg(m)
            o.apply_msg(m)
    B.flush()
    for j, (blobs, o, tail) in enumerate(cases):
        _same(B, j, o, f"case {j} after load + tail")
    # the tails the reference fails: equal before the failing op, "MergeTree insert failed" at it
    assert fails
    F = MergeTreeBatch(2 * len(fails), new_length_calc=new_mode)
    for j, (blobs, tail) in enumerate(fails):
        for q, n in ((2 * j, len(tail) - 1), (2 * j + 1, len(tail))):
            F[q].load(blobs, "loader")
            for m in tail[:n]:
                F[q].applyMsg(m)
    try:
        F.flush()
    except MergeTreeError:
        pass
    for j, (blobs, tail) in enumerate(fails):
        o = OracleDoc(new_length_calc=new_mode)
        o.load_v1(blobs, "loader")
        for m in tail[:-1]:
            o.apply_msg(m)
        _same(F, 2 * j, o, f"failing case {j} before its failing op")
        with pytest.raises(MergeTreeError, match="MergeTree insert failed"):  # (reads raise a document's error)
            F.map_range(2 * j + 1, 0, 1)


@pytest.mark.parametrize("new_mode", [False, True])
@pytest.mark.parametrize("chunk", [0, 300])
def test_long_documents_summarized_mid_collaboration(new_mode, chunk):
    """One client inserts past char 9,990 of a long text, every client removes and annotates there
    (tests/helpers.make_tail_log); SnapshotV1 summaries mid-log hold that client's segments, removed or not,
    above the MSN in their bodies.  Many such loads fail in the reference itself or leave deficits; every document
    must have the reference's outcome, each parameter set holds an equal outcome with deficits (the later ops
    advance the MSN: copyDown and recombination of the deficits), and the new length mode one with a phantom."""
    from helpers import make_tail_log
    from pyoracle import OracleDoc
    out = []
    # (seeds 40, 47, 48, 59: clean loads in the old length mode, where the first 16 all leave deficits or fail)
    for i in list(range(16)) + [40, 47, 48, 59]:
        text, msgs = make_tail_log(900 + i + 50 * int(new_mode), 1600, lag=24 + 8 * (i % 8), initial_len=9990, lo=9990,
                                   new_mode=new_mode, inserters=[0])
        cut = len(msgs) // 2 + 37 * (i % 8)
        a = OracleDoc(new_length_calc=new_mode, chunk_size=chunk)
        a.insert_text_local(0, text)
        a.start_collab("obs")
        for m in msgs[:cut]:
            a.apply_msg(m)
        blobs = [list(x) for x in a.summarize_v1()["blobs"]]
        r = _load_and_continue(blobs, msgs[cut:], new_mode, chunk)
        out.append((r, _phantoms(blobs)))
    print(f"long documents new_mode={new_mode} chunk={chunk}:", [r for r, _ in out])
    assert any(r == "deficit" for r, _ in out)
    if new_mode:  # (these seeds include equal outcomes with phantom body segments, counted on the oracle)
        assert any(r != "failed" and n > 0 for r, n in out)
