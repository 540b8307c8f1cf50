"""GPU parity: the HIP engine vs the reference's golden replay logs and vs the CPU oracle.

Bar: bit-exact.  Text after every one of the 1,920 fixture groups; canonical segment dumps (tree
shape, segment boundaries, seq/client/removal info, properties) and SnapshotV1 blobs byte-equal to
the oracle on synthetic multi-client logs in both length-calculation modes.
"""
import pytest

from helpers import first_diff, msg_from_compact, replay_fixtures

pytestmark = pytest.mark.gpu


def expected_alg_bytes(lb, i):
    """SURVEY 8(d) algorithmic bytes of document i, computed from the oracle's counters and the records."""
    import struct
    d = lb.docs[i]
    ops = lb.doc_ops_bytes(i)
    text_units = 0
    for k in range(d.n_ops):
        t, fl, _c, _s, _r, _m, _p1, p2, _pay, _pr = struct.unpack_from("<BBHIIIIIII", ops, 32 * k)
        if t == 0 and not fl & 0x42:  # text inserts (not markers / PermutationSegments)
            text_units += p2
    return 32 * d.ops_applied + 2 * text_units + 24 * d.segs_touched + 24 * d.final_segments + 2 * d.final_len


def _engine():
    from fluidframework_amd import MergeTreeBatch
    return MergeTreeBatch


def test_reference_replay_logs_text_every_group():
    """All 30 reference conflict-farm logs (client.replay.spec.ts) on one batch, 64 flushes."""
    fx = replay_fixtures()
    B = _engine()(len(fx))
    for i, (_, d) in enumerate(fx):
        c = B[i]
        c.insertTextLocal(0, d["initialText"])
        c.startOrUpdateCollaboration("A")
    ngroups = len(fx[0][1]["groups"])
    bad = []
    for g in range(ngroups):
        for i, (_, d) in enumerate(fx):
            for m in d["groups"][g]["msgs"]:
                B[i].applyMsg(msg_from_compact(m))
        B.flush()
        for i, (name, d) in enumerate(fx):
            if B[i].getText() != d["groups"][g]["resultText"]:
                bad.append((name, g))
    assert not bad, f"{len(bad)} mismatching (file, group) checkpoints, first: {bad[:5]}"


def _oracle_for_fixture(d):
    from pyoracle import OracleDoc
    o = OracleDoc()
    o.insert_text_local(0, d["initialText"])
    o.start_collab("A")
    for g in d["groups"]:
        for m in g["msgs"]:
            o.apply_msg(msg_from_compact(m))
    return o


def test_reference_replay_logs_segments_and_summary_match_oracle():
    fx = replay_fixtures()
    B = _engine()(len(fx))
    for i, (_, d) in enumerate(fx):
        B[i].insertTextLocal(0, d["initialText"])
        B[i].startOrUpdateCollaboration("A")
        for g in d["groups"]:
            for m in g["msgs"]:
                B[i].applyMsg(msg_from_compact(m))
    B.flush()
    for i, (name, d) in enumerate(fx):
        o = _oracle_for_fixture(d)
        gd, od = B.dump_segments(i), o.dump_segments()
        assert gd == od, f"{name}: segment dump differs: {first_diff(gd, od)}"
        assert B.digests(i, 1)[0] == o.digest(), f"{name}: state digest differs"
        gb, gs = B.summarize_v1(i)
        osum = o.summarize_v1()
        assert [list(x) for x in gb] == osum["blobs"], f"{name}: SnapshotV1 blobs differ"
        assert gs == osum["summary"], f"{name}: ISummaryTreeWithStats differs"


@pytest.mark.parametrize("new_mode", [False, True])
def test_synthetic_logs_bit_exact(new_mode):
    """64 synthetic docs x 2000 msgs, 8 clients, lag 128, groups + annotate, via binary records."""
    from pyloggen import LogBatch, make_cfg
    cfg = make_cfg(seed=11 + int(new_mode), n_ops=2000, new_length_calc=new_mode)
    lb = LogBatch(cfg, 0, 64)
    B = _engine()(lb.n, new_length_calc=new_mode)
    props = lb.props_json()
    ids = [B.intern_props(p) if p else 0 for p in props]
    assert ids == list(range(len(props))), "props ids must follow the generator table"
    for i in range(lb.n):
        tb = lb.doc_text_bytes(i)
        il = lb.docs[i].initial_len
        B.init_doc(i, tb[: il * 2].decode("utf-16-le"), "obs")
        for cid in lb.client_ids(i)[1:]:
            B.add_client(i, cid)
        # payload offsets in the generated records index the doc's text arena (initial text first)
        B.append_records(i, lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb)
    st = B.replay()
    assert st["errors"] == 0
    assert st["ops_applied"] == sum(lb.docs[i].ops_applied for i in range(lb.n))
    # state digests (GPU) == the oracle's, and the stats fold them
    dg = B.digests()
    assert dg == [lb.docs[i].digest for i in range(lb.n)]
    assert st["checksum"] == sum(dg) % (1 << 64)
    assert st["segments_final"] == sum(lb.docs[i].final_segments for i in range(lb.n))
    assert st["text_units_final"] == sum(lb.docs[i].final_len for i in range(lb.n))
    # roofline numerator: 32 B per op + 2 B per inserted text unit + 24 B per segment record
    # the oracle creates or modifies, + the final state write-back -- every term from the oracle
    assert st["bytes_alg"] == sum(expected_alg_bytes(lb, i) for i in range(lb.n))
    bad = [i for i in range(lb.n) if B.checksum(i) != lb.docs[i].checksum]
    if bad:
        from pyoracle import OracleDoc
        i = bad[0]
        o = OracleDoc(new_length_calc=new_mode)
        tb = lb.doc_text_bytes(i)
        il = lb.docs[i].initial_len
        if il:
            o.insert_text_local(0, tb[: il * 2].decode("utf-16-le"))
        o.start_collab("obs")
        for cid in lb.client_ids(i)[1:]:
            o.add_client(cid)
        o.apply_records(lb.doc_ops_bytes(i), lb.docs[i].n_ops, tb, props)
        pytest.fail(f"{len(bad)}/{lb.n} docs differ; doc {i}: {first_diff(B.dump_segments(i), o.dump_segments())}")
