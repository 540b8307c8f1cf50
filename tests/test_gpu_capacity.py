"""Slice capacities and the capacity retry (DESIGN.md §3 "HBM layout").

Large batches get tight per-document slices (caps_for's tight formula, ~1.4 MiB per 10k-record document instead
of ~4.5 MiB); a document whose first replay outgrows one of them is laid out again with that slice four times larger
and replayed from its pristine state, so tight caps never change a result.  MTB_CAPS=tight with a tiny
MTB_CAPS_SCALE forces many documents through the retry here.  Bar: every document's state digest (and a sample of
canonical dumps) equal to the oracle's, also after rewind + resident replay (the pristine snapshot follows the new
slices); with the retry disabled (MTB_CAP_RETRIES=0) an overflow is still reported as MTB_E_CAPACITY.
"""
import pytest

from helpers import first_diff, load_logbatch, records_to_msgs

pytestmark = pytest.mark.gpu


@pytest.fixture
def tiny_caps(monkeypatch):
    monkeypatch.setenv("MTB_CAPS", "tight")
    monkeypatch.setenv("MTB_CAPS_SCALE", "0.05")
    return monkeypatch


def _digests_equal(B, lb, docs):
    dg = B.digests()
    bad = [j for j in range(len(docs)) if dg[j] != lb.docs[docs[j]].digest]
    assert not bad, f"{len(bad)}/{len(docs)} documents differ from the oracle (first: {bad[:5]})"
    for j in range(0, len(docs), max(1, len(docs) // 6)):
        assert B.checksum(j) == lb.docs[docs[j]].checksum


@pytest.mark.parametrize("n_docs,n_ops", [(48, 1500), (4200, 160)])
def test_capacity_retry_gives_the_oracle_result(tiny_caps, n_docs, n_ops):
    """(4,200 documents run the ticket-scheduled kernel, 48 the few-document one.)"""
    from fluidframework_amd import MergeTreeBatch
    from pyloggen import LogBatch, make_cfg
    lb = LogBatch(make_cfg(seed=611 + n_docs, n_ops=n_ops), 0, n_docs)
    B = MergeTreeBatch(n_docs)
    docs = load_logbatch(B, lb)
    st = B.replay()
    assert st["errors"] == 0
    li = B.launch_info()
    assert li["cap_retries"] >= 1, "the tiny caps did not force a capacity retry"
    _digests_equal(B, lb, docs)
    assert st["checksum"] == sum(lb.docs[u].digest for u in docs) % (1 << 64)
    # rewind restores every document into its (re-laid-out) slices; the resident replay fits without a retry
    B.rewind()
    st2 = B.replay_resident()
    assert st2["errors"] == 0 and st2["checksum"] == st["checksum"]
    _digests_equal(B, lb, docs)


def test_capacity_overflow_without_retry_reports_capacity(tiny_caps):
    from fluidframework_amd import MergeTreeBatch
    from fluidframework_amd.client import MergeTreeError
    from pyloggen import LogBatch, make_cfg
    tiny_caps.setenv("MTB_CAP_RETRIES", "0")
    lb = LogBatch(make_cfg(seed=613, n_ops=1500), 0, 8)
    B = MergeTreeBatch(8)
    load_logbatch(B, lb)
    with pytest.raises(MergeTreeError) as ei:
        B.replay()
    assert ei.value.code == -7 and "capacity" in str(ei.value)


def test_capacity_retry_of_loaded_documents(tiny_caps):
    """Summaries loaded and continued in one replay: the retry restores the loaded header tree (its window lists
    and aux words included) before replaying the body and the ops again."""
    from fluidframework_amd import MergeTreeBatch
    from pyoracle import OracleDoc
    from pyloggen import LogBatch, make_cfg
    lb = LogBatch(make_cfg(seed=617, n_ops=1200), 0, 12)
    props = lb.props_json()
    B = MergeTreeBatch(lb.n)
    oracles = []
    for i in range(lb.n):
        tb = lb.doc_text_bytes(i)
        il = lb.docs[i].initial_len
        msgs = records_to_msgs(lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb, props, lb.client_ids(i))
        cut = len(msgs) // 2
        a = OracleDoc()
        a.insert_text_local(0, tb[: il * 2].decode("utf-16-le"))
        a.start_collab("obs")
        for m in msgs[:cut]:
            a.apply_msg(m)
        blobs = [list(x) for x in a.summarize_v1()["blobs"]]
        B[i].load(blobs, "obs")
        o = OracleDoc()
        o.load_v1(blobs, "obs")
        for m in msgs[cut:]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
    B.flush()
    assert B.launch_info()["cap_retries"] >= 1
    for i, o in enumerate(oracles):
        gd, od = B.dump_segments(i), o.dump_segments()
        assert gd == od, f"doc {i}: segment dump differs: {first_diff(gd, od)}"
        assert B.text(i) == o.get_text()
