"""GPU parity of the SharedMatrix PermutationVector path.

Each matrix is two PermutationVector documents replayed by one 128-lane workgroup (wave 0 rows, wave 1
cols); a remote setCell meets at a workgroup barrier so each vector allocates its handle only when both
adjusted positions survive (matrix.ts:668-676).  Bar: bit-exact against the oracle's restatement
(oracle/mt_oracle.cpp MatrixDoc): canonical segment dumps with PermutationSegment [length, start] and the
handle table, and PermutationVector.summarize (SnapshotV1 segments + handleTable blob), in both length
modes, on generated op streams (row/col insert/remove of 1..8, setCell, lagging refSeqs).
The reference holds no golden matrix data, so the oracle here is parity-unpinned beyond code reading.
"""
import pytest

from helpers import first_diff, make_matrix_log

pytestmark = pytest.mark.gpu


def _check(B, m, o, what, cells=True):
    if cells:  # SharedMatrix.summarize: rows / cols PermutationVector summaries + the cells blob
        gb, gs = B.matrix_summarize(m)
        osum = o.summarize()
        assert [list(x) for x in gb] == osum["blobs"], f"{what}: matrix summary blobs differ"
        assert gs == osum["summary"], f"{what}: matrix summary tree differs"
    for name, doc, od in (("rows", 2 * m, o.rows), ("cols", 2 * m + 1, o.cols)):
        gd, odd = B.dump_segments(doc), od.dump_segments()
        assert gd == odd, f"{what} {name}: dump differs: {first_diff(gd, odd)}"
        gb, gs = B.summarize_v1(doc)
        osum = od.summarize_v1()
        assert [list(x) for x in gb] == osum["blobs"], f"{what} {name}: summary blobs differ"
        assert gs == osum["summary"], f"{what} {name}: summary tree differs"


@pytest.mark.parametrize("new_mode", [False, True])
def test_generated_matrix_logs_match_oracle(new_mode):
    from fluidframework_amd import MatrixBatch
    from pyoracle import OracleMatrix
    n = 24
    logs = [make_matrix_log(100 + 7 * i + int(new_mode), 300 + 25 * i, n_clients=2 + i % 5, lag=4 + 3 * (i % 7),
                            p_set=0.2 + 0.05 * (i % 9), new_mode=new_mode) for i in range(n)]
    B = MatrixBatch(n, new_length_calc=new_mode)
    oracles = []
    for i, msgs in enumerate(logs):
        B[i].startOrUpdateCollaboration("obs")
        o = OracleMatrix(new_length_calc=new_mode)
        o.start_collab("obs")
        half = len(msgs) // 2
        for m in msgs[:half]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append((o, msgs[half:]))
    B.flush()  # first half, then check, then the rest (the same records path twice)
    for i, (o, _) in enumerate(oracles):
        _check(B, i, o, f"matrix {i} (half)")
    for i, (o, rest) in enumerate(oracles):
        for m in rest:
            B[i].applyMsg(m)
            o.apply_msg(m)
    B.flush()
    for i, (o, _) in enumerate(oracles):
        _check(B, i, o, f"matrix {i}")
        # getCell over the whole observer view (matrix.ts:173-189)
        nr, nc = o.rows.get_length(), o.cols.get_length()
        for r in range(0, nr, max(1, nr // 12)):
            for c in range(0, nc, max(1, nc // 12)):
                assert B.get_cell(i, r, c) == o.get_cell(r, c), f"matrix {i} cell ({r}, {c})"


def test_rewind_restores_handle_tables():
    """Rewind + resident replay of a matrix batch gives the same vectors (handle tables included)."""
    from fluidframework_amd import MatrixBatch
    from pyoracle import OracleMatrix
    msgs = make_matrix_log(5, 400, n_clients=3)
    B = MatrixBatch(1)
    B[0].startOrUpdateCollaboration("obs")
    o = OracleMatrix()
    o.start_collab("obs")
    for m in msgs:
        B[0].applyMsg(m)
        o.apply_msg(m)
    B.flush()
    _check(B, 0, o, "matrix")
    first = (B.dump_segments(0), B.dump_segments(1))
    B.rewind()
    B.replay_resident()
    assert (B.dump_segments(0), B.dump_segments(1)) == first
    _check(B, 0, o, "matrix after rewind")


@pytest.mark.parametrize("new_mode", [False, True])
def test_generated_matrix_records_match_oracle_checksums(new_mode):
    """64 generated matrices x 3,000 messages through the pre-packed record path (mtb_append_ops): each
    vector's canonical dump checksum equals the generator's oracle."""
    from fluidframework_amd import MatrixBatch
    from pyloggen import MatrixLogBatch, make_cfg
    lb = MatrixLogBatch(make_cfg(seed=77 + int(new_mode), n_ops=3000, lag=48, new_length_calc=new_mode), 0, 64)
    B = MatrixBatch(lb.n, new_length_calc=new_mode)
    lb.intern_values(B)
    for i in range(lb.n):
        B.init_matrix(i, "obs")
        for v in (0, 1):
            for cid in lb.client_ids(i, v)[1:]:
                B.add_client(2 * i + v, cid)
            B.append_records(2 * i + v, lb.ops_bytes(i, v), lb.mats[i].n_ops[v], b"")
    st = B.replay()
    assert st["errors"] == 0
    bad = [(i, v) for i in range(lb.n) for v in (0, 1) if B.checksum(2 * i + v) != lb.mats[i].checksum[v]]
    assert not bad, f"{len(bad)} vectors differ, first {bad[:4]}"


@pytest.mark.parametrize("new_mode", [False, True])
def test_matrix_load_mid_stream_then_continue(new_mode, chunk_size=0):
    """SharedMatrix.loadCore (matrix.ts:611-634) on the engine: an oracle summary taken mid-stream is loaded
    (rows / cols handle tables + segments, cells) and the rest of the log replayed; summaries and getCell
    equal the oracle that loaded the same summary."""
    from fluidframework_amd import MatrixBatch
    from pyoracle import OracleMatrix
    n = 12
    B = MatrixBatch(n, new_length_calc=new_mode, chunk_size=chunk_size)
    oracles = []
    bodies = 0
    for i in range(n):
        msgs = make_matrix_log(700 + 3 * i + int(new_mode), 600 + 20 * i, n_clients=2 + i % 4, lag=3 + 2 * (i % 6),
                               new_mode=new_mode)
        src = OracleMatrix(new_length_calc=new_mode, chunk_size=chunk_size)
        src.start_collab("obs")
        half = len(msgs) // 2
        for m in msgs[:half]:
            src.apply_msg(m)
        blobs = src.summarize()["blobs"]
        bodies += sum(1 for p, _ in blobs if "/body_" in p)
        o = OracleMatrix(new_length_calc=new_mode, chunk_size=chunk_size)
        o.load(blobs, "obs")
        B[i].load(blobs, "obs")
        for m in msgs[half:]:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
    B.flush()
    for i, o in enumerate(oracles):
        _check(B, i, o, f"loaded matrix {i}")
        nr, nc = o.rows.get_length(), o.cols.get_length()
        for r in range(0, nr, max(1, nr // 10)):
            for c in range(0, nc, max(1, nc // 10)):
                assert B.get_cell(i, r, c) == o.get_cell(r, c), f"matrix {i} cell ({r}, {c})"
    assert (bodies > 0) == (chunk_size > 0)


@pytest.mark.parametrize("new_mode", [False, True])
def test_matrix_load_body_chunks_at_quiescence(new_mode):
    """PermutationVector summaries with body chunks (permutationvector.ts:310-325, chunkSize 5) loaded on the
    engine (mtb_load_perm_kernel appends the bodies, snapshotLoader.ts:169-220): each vector summarized with
    the runtime's MSN = lastSequenceNumber (Client.summarize, client.ts:966-1005), the matrix loaded, then a
    continuation generated against the loaded state; dumps, summaries and the getCell grid equal the oracle
    that loaded the same summary.  (Mid-stream summaries whose header holds segments above the MSN can make
    the reference's body insert fail, as the oracle and engine both reproduce in test_gpu_load.py.)"""
    import json as _json
    from fluidframework_amd import MatrixBatch
    from pyoracle import OracleMatrix
    n, cs = 8, 5
    B = MatrixBatch(n, new_length_calc=new_mode, chunk_size=cs)
    oracles = []
    bodies = 0
    for i in range(n):
        msgs = make_matrix_log(900 + 5 * i + int(new_mode), 400 + 40 * i, n_clients=2 + i % 3, lag=2 + i % 4,
                               new_mode=new_mode)
        src = OracleMatrix(new_length_calc=new_mode, chunk_size=cs)
        src.start_collab("obs")
        for m in msgs:
            src.apply_msg(m)
        last = msgs[-1]["sequenceNumber"]
        blobs = []
        for name, vec in (("rows", src.rows), ("cols", src.cols)):
            for p, c in vec.summarize_v1(last, last)["blobs"]:
                blobs.append([f"{name}/{p}", c])
        blobs += [b for b in src.summarize()["blobs"] if b[0] == "cells"]
        bodies += sum(1 for p, _ in blobs if "/body_" in p)
        o = OracleMatrix(new_length_calc=new_mode, chunk_size=cs)
        o.load(blobs, "obs")
        gen = OracleMatrix(new_length_calc=new_mode, chunk_size=cs)
        gen.load(blobs, "obs")
        rest = make_matrix_log(950 + i, 150, n_clients=2 + i % 3, lag=2, new_mode=new_mode, start=(gen, last))
        B[i].load(blobs, "obs")
        for m in rest:
            B[i].applyMsg(m)
            o.apply_msg(m)
        oracles.append(o)
    B.flush()
    assert bodies > 0
    for i, o in enumerate(oracles):
        _check(B, i, o, f"loaded matrix {i}")
        nr, nc = o.rows.get_length(), o.cols.get_length()
        for r in range(0, nr, max(1, nr // 8)):
            for c in range(0, nc, max(1, nc // 8)):
                assert B.get_cell(i, r, c) == o.get_cell(r, c), f"matrix {i} cell ({r}, {c})"


@pytest.mark.parametrize("new_mode", [False, True])
def test_reference_conflict_kats_gpu(new_mode):
    """matrix.spec.ts:349-607 two-client conflict cases (tests/matrix_kats.py) on the engine: each case's
    grid equals the spec's literal, and dumps / summaries equal the oracle's (all cases in one batch)."""
    import json
    from fluidframework_amd import MatrixBatch
    from matrix_kats import CASES, case_messages, grid
    from test_matrix_kats import oracle_grid
    B = MatrixBatch(len(CASES), new_length_calc=new_mode)
    logs = [case_messages(c[2]) for c in CASES]
    for i, msgs in enumerate(logs):
        B[i].startOrUpdateCollaboration("observer")
        for m in msgs:
            B[i].applyMsg(m)
    B.flush()
    for i, (name, line, _, expected) in enumerate(CASES):
        og, o = oracle_grid(logs[i], new_mode)
        gg = grid(B.length(2 * i), B.length(2 * i + 1), lambda r, c: B[i].getCell(r, c))
        assert gg == og, f"matrix.spec.ts:{line} {name!r}: engine grid {gg} != oracle {og}"
        if expected is not None:
            assert gg == expected, f"matrix.spec.ts:{line} {name!r}"
        _check(B, i, o, name)


def test_matrix_bench_parity_definition():
    """bench_matrix.py's total parity on a small batch: every vector's GPU state digest equals the generator
    oracle's Doc::digest and every matrix's summary fingerprint (mtb_blob_list_fnv of
    SharedMatrix.summarizeCore) equals the oracle's (oracle/loggen.cpp summary_fnv)."""
    from fluidframework_amd import MatrixBatch
    from pyloggen import MatrixLogBatch, make_cfg
    cfg = make_cfg(seed=77, n_clients=6, n_ops=1500, lag=32, pct_set=40)
    lb = MatrixLogBatch(cfg, 0, 24)
    B = MatrixBatch(lb.n)
    lb.intern_values(B)
    for j in range(lb.n):
        B.init_matrix(j, "obs")
        for v in (0, 1):
            for cid in lb.client_ids(j, v)[1:]:
                B.add_client(2 * j + v, cid)
            B.append_records(2 * j + v, lb.ops_bytes(j, v), lb.mats[j].n_ops[v], b"")
    st = B.replay()
    assert st["errors"] == 0
    dig = B.digests()
    for j in range(lb.n):
        assert (dig[2 * j], dig[2 * j + 1]) == (lb.mats[j].digest[0], lb.mats[j].digest[1]), j
        assert B.matrix_summary_fnv(j) == lb.mats[j].summary_fnv, j
