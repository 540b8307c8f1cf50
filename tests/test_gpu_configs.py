"""GPU parity on scaled versions of every BASELINE.json configuration.

* configs[1] (10k docs x 8 clients x 10k ops) runs at full size in bench.py, which compares every
  document's GPU state digest with the generator's oracle digest; here a 64-document slice.
* configs[2] (doc-hash sharding): two shards built with shard_docs replay on device 0 as two batches;
  the union of their per-document digests equals one unsharded batch and the oracle.
* configs[3] (one long document, 64 clients, lag 512): a 100k-char initial text and 30k messages.
* configs[4] (annotate-heavy SharedString half: 60 % annotate, 10 property keys), both length modes.
Bar: bit-exact (state digest and the FNV-1a checksum of the canonical segment dump equal the oracle's).
"""
import pytest

from helpers import load_logbatch

pytestmark = pytest.mark.gpu


def _batch(n, new_mode=False):
    from fluidframework_amd import MergeTreeBatch
    return MergeTreeBatch(n, new_length_calc=new_mode)


def _check(B, lb, docs, st):
    assert st["errors"] == 0
    dg = B.digests()
    want = [lb.docs[u].digest for u in docs]
    bad = [j for j in range(len(docs)) if dg[j] != want[j]]
    assert not bad, f"{len(bad)}/{len(docs)} documents' state digests differ from the oracle (first: {bad[:5]})"
    assert st["checksum"] == sum(want) % (1 << 64)
    for j in range(0, len(docs), max(1, len(docs) // 8)):
        assert B.checksum(j) == lb.docs[docs[j]].checksum


def test_cfg4_long_document_scaled():
    """configs[3] scaled: 100k-char initial text, 64 writer clients, refSeq lag 512, 30k messages."""
    from pyloggen import LogBatch, make_cfg
    cfg = make_cfg(seed=404, n_clients=64, n_ops=30000, lag=512, initial_len=100000)
    lb = LogBatch(cfg, 0, 1)
    B = _batch(1)
    docs = load_logbatch(B, lb)
    st = B.replay()
    _check(B, lb, docs, st)
    assert st["ops_applied"] == lb.docs[0].ops_applied


def test_cfg3_document_hash_shards_partition_the_batch():
    """configs[2] shape: documents sharded by hash(doc) mod 2 (fluidframework_amd.sharding) replay as two
    batches whose per-document digests are exactly the unsharded batch's, and whose checksum sums add up."""
    from fluidframework_amd.sharding import shard_docs
    from pyloggen import LogBatch, make_cfg
    total = 96
    cfg = make_cfg(seed=303, n_ops=1500)
    lb = LogBatch(cfg, 0, total)
    whole = _batch(total)
    load_logbatch(whole, lb)
    st_whole = whole.replay()
    _check(whole, lb, list(range(total)), st_whole)
    dig_whole = whole.digests()
    seen = {}
    sums = 0
    for r in range(2):
        mine = shard_docs(total, 2, r)
        S = _batch(len(mine))
        load_logbatch(S, lb, mine)
        st = S.replay()
        assert st["errors"] == 0
        for j, g in enumerate(S.digests()):
            seen[mine[j]] = g
        sums += st["checksum"]
    assert sorted(seen) == list(range(total))
    assert [seen[g] for g in range(total)] == dig_whole
    assert sums % (1 << 64) == st_whole["checksum"]


@pytest.mark.parametrize("new_mode", [False, True])
def test_cfg5_annotate_heavy_strings(new_mode):
    """configs[4], SharedString half: 60 % annotate over 10 property keys, 20 % insert, 20 % remove."""
    from pyloggen import LogBatch, make_cfg
    cfg = make_cfg(seed=505 + int(new_mode), n_ops=2000, pct_insert=20, pct_remove=20, annotate_keys=10,
                   new_length_calc=new_mode)
    lb = LogBatch(cfg, 0, 48)
    B = _batch(lb.n, new_mode)
    docs = load_logbatch(B, lb)
    st = B.replay()
    _check(B, lb, docs, st)


def test_cfg2_slice_full_length_logs():
    """configs[1] slice: 64 documents x 10,000 messages (the bench's per-document length), 8 clients; the
    north star's SnapshotV1 summaries of every document byte-equal to the oracle's (batched summarize)."""
    from pyloggen import LogBatch, make_cfg
    cfg = make_cfg(seed=202, n_ops=10000)
    lb = LogBatch(cfg, 0, 64)
    B = _batch(lb.n)
    docs = load_logbatch(B, lb)
    st = B.replay()
    _check(B, lb, docs, st)
    fps = B.summarize_v1_many(list(range(lb.n)), threads=8, fingerprints=True)
    bad = [j for j in range(lb.n) if fps[j] != lb.docs[j].summary_fnv]
    assert not bad, f"{len(bad)}/{lb.n} SnapshotV1 summaries differ from the oracle's (first: {bad[:5]})"
    full = B.summarize_v1_many([3, 17], threads=2)
    assert [list(map(list, full[0][0])), full[0][1]] == [list(map(list, B.summarize_v1(3)[0])), B.summarize_v1(3)[1]]
    assert full[1][0] == B.summarize_v1(17)[0]


def test_multi_shard_batch_on_one_device(monkeypatch):
    """The multi-device front end (mtb_multi.cpp) with 3 shards on device 0 (MTB_SHARDS_PER_DEVICE): the
    shards replay at once from three host threads (three streams); every document's digest, the merged
    stats and the batched summaries equal the oracle's, also after rewind + resident replay."""
    from fluidframework_amd import MergeTreeBatch
    from pyloggen import LogBatch, make_cfg
    cfg = make_cfg(seed=707, n_ops=1500)
    lb = LogBatch(cfg, 0, 40)
    monkeypatch.setenv("MTB_SHARDS_PER_DEVICE", "3")
    B = MergeTreeBatch(lb.n)
    monkeypatch.delenv("MTB_SHARDS_PER_DEVICE")
    docs = load_logbatch(B, lb)
    st = B.replay()
    _check(B, lb, docs, st)
    assert st["ops_applied"] == sum(d.ops_applied for d in lb.docs)
    fps = B.summarize_v1_many(list(range(lb.n)), threads=6, fingerprints=True)
    assert fps == [lb.docs[j].summary_fnv for j in range(lb.n)]
    B.rewind()
    st2 = B.replay_resident()
    assert st2["checksum"] == st["checksum"] and st2["ops_applied"] == st["ops_applied"]
    assert B.digests() == [lb.docs[j].digest for j in range(lb.n)]
    # the bench's timed form: no digest pass in the replay, one afterwards (mtb_refresh_digests)
    B.rewind()
    st3 = B.replay_resident(digests=False)
    assert st3["checksum"] == 0 and st3["ops_applied"] == st["ops_applied"]
    with pytest.raises(Exception, match="no digests"):
        B.digests()
    fin = B.refresh_digests()
    assert fin["checksum"] == st["checksum"] and st3["bytes_alg"] + fin["bytes_alg"] == st2["bytes_alg"]
    assert B.digests() == [lb.docs[j].digest for j in range(lb.n)]


def _prefix_digest(lb, u, m):
    """the oracle's digest of log u's first m records (an observer set up as load_logbatch sets up the engine)"""
    import sys
    from pyoracle import OracleDoc
    tb = lb.doc_text_bytes(u)
    o = OracleDoc()
    o.insert_text_local(0, tb[: lb.docs[u].initial_len * 2].decode("utf-16-le"))
    o.start_collab("obs")
    for cid in lb.client_ids(u)[1:]:
        o.add_client(cid)
    o.apply_records(lb.doc_ops_bytes(u)[: 32 * m], m, tb, lb.props_json())
    return o.digest()


def _message_cut(lb, u, frac):
    """a record count at a message boundary (the record before it carries the LAST flag) near frac"""
    ob = lb.doc_ops_bytes(u)
    m = int(lb.docs[u].n_ops * frac)
    while m > 0 and not (ob[32 * (m - 1) + 1] & 1):
        m -= 1
    return m


@pytest.mark.parametrize("chunks,queues,spins", [(None, None, None), ("16", None, None), ("3", "1", None),
                                                 (None, None, "0"), ("16", "1", "40")])
def test_scheduled_replay_more_documents_than_wave_slots(monkeypatch, chunks, queues, spins):
    """More documents than the device's resident replay waves runs ticket-scheduled replay -- one ticket per
    workgroup (mtb_replay_tick_kernel), documents advanced chunk by chunk in round-robin: 4,608 documents with ragged record counts --
    whole 300-message logs, message-boundary prefixes of them, and documents with no records -- every
    state digest equal to the oracle's, for the default shrinking-chunk plan and for 16 and 3 equal chunks
    per document (MTB_CHUNKS), per-XCD ticket queues and one global queue (MTB_SCHED_QUEUES=1), and with
    the ticket waits bounded so low that the scheduler aborts (MTB_SCHED_SPINS): the finish kernel then
    replays the rest of every document and the results are the same."""
    monkeypatch.delenv("MTB_CHUNK_PLAN", raising=False)
    monkeypatch.delenv("MTB_SCHED", raising=False)
    for var, val in (("MTB_CHUNKS", chunks), ("MTB_SCHED_QUEUES", queues), ("MTB_SCHED_SPINS", spins)):
        if val is None:
            monkeypatch.delenv(var, raising=False)
        else:
            monkeypatch.setenv(var, val)
    B, want, slots = _ragged_batch()
    st = B.replay()
    assert st["errors"] == 0
    li = B.launch_info()
    assert li["kernel"] == "mtb_replay_tick_kernel" and li["wave_slots"] == slots, li
    if spins == "0":
        assert li["aborted"], li  # every hand-over wait gives up at once
    dg = B.digests()
    n = len(want)
    bad = [j for j in range(n) if dg[j] != want[j]]
    assert not bad, f"{len(bad)}/{n} documents' digests differ from the oracle (first: {bad[:5]})"


@pytest.mark.parametrize("chunks", [None, "1", "3", "7"])
def test_pass_replay_more_documents_than_wave_slots(monkeypatch, chunks):
    """Passes (MTB_SCHED=passes, mtb_replay_pass_kernel) for more documents than resident replay waves.  The
    documents' chunks, chunk-major, are cut into launches of whole rounds of the wave slots, at most one chunk
    per document each, so the launch boundaries order every document's chunks.  The same 4,608 ragged
    documents as the ticket test: every digest equal to the oracle's, for the chosen chunk count and for 1, 3
    and 7 chunks per document (MTB_PASS_CHUNKS); the pass count follows the cut."""
    monkeypatch.setenv("MTB_SCHED", "passes")
    if chunks is None:
        monkeypatch.delenv("MTB_PASS_CHUNKS", raising=False)
    else:
        monkeypatch.setenv("MTB_PASS_CHUNKS", chunks)
    B, want, slots = _ragged_batch()
    n = len(want)
    st = B.replay()
    assert st["errors"] == 0
    li = B.launch_info()
    assert li["kernel"] == "mtb_replay_pass_kernel" and li["wave_slots"] == slots, li
    per = max(1, n // slots) * slots
    assert li["passes"] == -(-li["chunks"] * n // per), li
    if chunks is not None:
        assert li["chunks"] == int(chunks)
    dg = B.digests()
    bad = [j for j in range(n) if dg[j] != want[j]]
    assert not bad, f"{len(bad)}/{n} documents' digests differ from the oracle (first: {bad[:5]})"


def _ragged_batch():
    """slots + slots / 8 documents with ragged record counts -- whole 300-message logs, message-boundary
    prefixes of them, and documents with no records -- and the oracle's digest each should end with."""
    import torch
    from pyloggen import LogBatch, make_cfg
    lb = LogBatch(make_cfg(seed=606, n_ops=300), 0, 48)
    slots = torch.cuda.get_device_properties(0).multi_processor_count * 16
    n = slots + slots // 8  # more documents than resident replay waves
    B = _batch(n)
    props = lb.props_json()
    assert [B.intern_props(p) if p else 0 for p in props] == list(range(len(props)))
    want = []
    prefix = {}
    for j in range(n):
        u = (j * 7) % lb.n
        tb = lb.doc_text_bytes(u)
        B.init_doc(j, tb[: lb.docs[u].initial_len * 2].decode("utf-16-le"), "obs")
        for cid in lb.client_ids(u)[1:]:
            B.add_client(j, cid)
        if j % 211 == 5:
            m = 0
        elif j % 97 == 3:
            m = _message_cut(lb, u, 0.1 + 0.8 * ((j // 97) % 5) / 5)
        else:
            m = lb.docs[u].n_ops
        if m:
            B.append_records(j, lb.doc_ops_bytes(u)[: 32 * m], m, tb)
        if m == lb.docs[u].n_ops:
            want.append(lb.docs[u].digest)
        else:
            if (u, m) not in prefix:
                prefix[(u, m)] = _prefix_digest(lb, u, m)
            want.append(prefix[(u, m)])
    return B, want, slots
