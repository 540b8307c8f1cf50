"""Benchmark of SURVEY.md 8(f) rank 2 / cfg5: SharedMatrix PermutationVector replay.

Workload: per GPU 10,000 SharedMatrix observers, 8 writer clients, 5,000 sequenced messages per matrix:
row/col inserts and removes of 1..8 (60/40 when not a setCell) and 40% setCell (remote cell writes that
adjust (row, col) into the observer's view and allocate storage handles), refSeq lag U{0..64}, legacy
length calculation.  Each matrix is one 128-lane workgroup (wave 0 = rows vector, wave 1 = cols vector)
of mtb_matrix_kernel.  One step = rewind + replay of every matrix with records resident in HBM.

value = sequenced messages applied per second (vector ops + setCells).  The roofline line is for
mtb_matrix_kernel with the same algorithmic-bytes rule as bench.py (32 B per record + 24 B per segment
record created or modified).  cpu_baseline: the C++ oracle replays a bounded sample on the host cores.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBPS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrices", type=int, default=10000)
    ap.add_argument("--replicas", type=int, default=10)
    ap.add_argument("--msgs", type=int, default=5000)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--lag", type=int, default=64)
    ap.add_argument("--pct-set", type=int, default=40)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=400)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=20260303)
    args = ap.parse_args()

    from fluidframework_amd import MatrixBatch
    from pyloggen import MatrixLogBatch, make_cfg

    reps = max(1, args.replicas)
    n_unique = (args.matrices + reps - 1) // reps
    cfg = make_cfg(seed=args.seed, n_clients=args.clients, n_ops=args.msgs, lag=args.lag, pct_set=args.pct_set)
    t0 = time.time()
    lb = MatrixLogBatch(cfg, 0, n_unique)
    t_gen = time.time() - t0
    B = MatrixBatch(args.matrices)
    opsb = [[lb.ops_bytes(u, v) for v in (0, 1)] for u in range(n_unique)]
    ids = [[lb.client_ids(u, v) for v in (0, 1)] for u in range(n_unique)]
    t0 = time.time()
    for j in range(args.matrices):
        u = j // reps
        B.init_matrix(j, "obs")
        for v in (0, 1):
            for cid in ids[u][v][1:]:
                B.add_client(2 * j + v, cid)
            B.append_records(2 * j + v, opsb[u][v], lb.mats[u].n_ops[v], b"")
    st = B.replay()
    t_load = time.time() - t0
    if st["errors"]:
        raise SystemExit(f"replay errors: {st['errors']}")

    def step():
        B.rewind()
        return B.replay_resident()

    for _ in range(args.warmup):
        step()
    times, kms = [], []
    last = None
    for _ in range(args.steps):
        t0 = time.perf_counter()
        last = step()
        times.append(time.perf_counter() - t0)
        kms.append(last["kernel_ms"])
    el = sum(times) / len(times)
    km = sum(kms) / len(kms)
    bad = 0
    sample = list(range(0, args.matrices, max(1, args.matrices // 32)))[:32]
    for j in sample:
        u = j // reps
        bad += sum(B.checksum(2 * j + v) != lb.mats[u].checksum[v] for v in (0, 1))
    msgs = sum(lb.mats[j // reps].n_msgs for j in range(args.matrices))
    sets = sum(lb.mats[j // reps].n_sets for j in range(args.matrices))
    records = sum(lb.mats[j // reps].n_ops[v] for j in range(args.matrices) for v in (0, 1))
    alg = last["bytes_alg"] + 32 * (records - last["ops_applied"])  # SETCELL records are read too
    cpu = None
    if not args.no_cpu:
        k = min(args.cpu_sample, n_unique)
        thr = min(16, os.cpu_count() or 1)
        secs, cbad = lb.cpu_replay(n=k, threads=thr)
        cm = sum(lb.mats[u].n_msgs for u in range(k))
        cpu = {"value": round(cm / secs, 1), "unit": "msgs/s", "cores": thr, "kind": "port",
               "sample": f"{k} matrices x {args.msgs} msgs ({cm} msgs) of the same logs, C++ oracle (oracle/), "
                         f"{thr} threads, {secs:.2f}s, {cbad} mismatches"}
    out = {
        "metric": "SharedMatrix sequenced messages applied/sec (rows+cols PermutationVectors + setCell handles)",
        "value": round(msgs / el, 1),
        "unit": "msgs/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": f"synthetic: {n_unique} generated matrix logs, each replayed as {reps} matrices",
        "config": {"workload": f"matrix-10k: {args.matrices} SharedMatrix observers x {args.clients} clients x "
                               f"{args.msgs} msgs, {args.pct_set}% setCell, row/col counts 1..8, lag {args.lag}",
                   "msgs_per_step": msgs, "setcells_per_step": sets, "records_per_step": records},
        "roofline": {"bound": "hbm", "achieved": round(alg / (km * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(alg / (km * 1e-3) / 1e9 / HBM_PEAK_GBPS, 6), "traffic": None,
                     "kernel": "mtb_matrix_kernel", "kernel_ms": round(km, 3), "alg_bytes_per_launch": alg},
        "cpu_baseline": cpu,
        "parity": {"sampled_vectors": 2 * len(sample), "mismatches": bad},
        "timing": {"generate_s": round(t_gen, 2), "load_and_first_replay_s": round(t_load, 2)},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
