"""Benchmark of SURVEY.md 8(f) rank 2 / cfg5: SharedMatrix PermutationVector replay.

Workload: per GPU 10,000 SharedMatrix observers, 8 writer clients, 5,000 sequenced messages per matrix:
row/col inserts and removes of 1..8 (60/40 when not a setCell) and 40% setCell (remote cell writes that
adjust (row, col) into the observer's view and allocate storage handles), refSeq lag U{0..64}, legacy
length calculation.  Each matrix is one 128-lane workgroup (wave 0 = rows vector, wave 1 = cols vector)
of mtb_matrix_kernel.  One step = rewind + replay of every matrix with records resident in HBM.

value = sequenced messages applied per second (vector ops + setCells).  The roofline line is for
mtb_matrix_kernel with the same algorithmic-bytes rule as bench.py (32 B per record + 24 B per segment
record created or modified); `traffic` = FETCH_SIZE x 2 + WRITE_SIZE of one launch from two rocprofv3 --pmc
child runs (as bench.py).  cpu_baseline: the C++ oracle replays a bounded sample on the host cores.

parity (every matrix, one unique log each by default): both vectors' GPU state digests against the
generator oracle's (Doc::digest), and the FNV-1a of every matrix's SharedMatrix summary blobs (rows / cols
PermutationVector summaries, handle tables, cells) against the oracle's summary of the same log.
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


def _traffic(args):
    """HBM bytes of one mtb_matrix_kernel launch: FETCH_SIZE (x2, the gfx950 correction) and WRITE_SIZE from
    two separate rocprofv3 --pmc child runs of this benchmark (1 step), as bench.py measures the string kernel."""
    import csv
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, None
    vals = {}
    with tempfile.TemporaryDirectory(prefix="mtb_pmc_") as td:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(td, counter.lower())
            cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", out, "-o", counter.lower(), "--",
                   sys.executable, os.path.abspath(__file__), "--no-cpu", "--no-parity", "--traffic", "off", "--steps",
                   "1", "--warmup", "0", "--matrices", str(args.matrices), "--replicas", str(args.replicas), "--msgs",
                   str(args.msgs), "--clients", str(args.clients), "--lag", str(args.lag), "--pct-set",
                   str(args.pct_set), "--seed", str(args.seed)]
            try:
                subprocess.run(cmd, env=dict(os.environ, MTB_IN_PMC="1"), stdout=subprocess.DEVNULL, timeout=900,
                               check=True)
            except Exception:
                return None, None
            per = {}
            for root, _, files in os.walk(out):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        for r in csv.DictReader(open(os.path.join(root, f))):
                            if "mtb_matrix_kernel" in r["Kernel_Name"]:
                                per[int(r["Dispatch_Id"])] = per.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
            if not per:
                return None, None
            vals[counter] = per[max(per)]
    fetch_b, write_b = 2.0 * vals["FETCH_SIZE"] * 1024.0, vals["WRITE_SIZE"] * 1024.0
    return round(fetch_b + write_b), {"fetch_size_kib": vals["FETCH_SIZE"], "write_size_kib": vals["WRITE_SIZE"],
                                      "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
                                      "note": "last mtb_matrix_kernel launch; FETCH_SIZE doubled per the gfx950 correction"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrices", type=int, default=10000)
    ap.add_argument("--replicas", type=int, default=1)
    ap.add_argument("--msgs", type=int, default=5000)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--lag", type=int, default=64)
    ap.add_argument("--pct-set", type=int, default=40)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=400)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=20260303)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--traffic", choices=["auto", "off"], default="auto")
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
    lb.intern_values(B)
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
    bad_dig = bad_sum = 0
    t_par = time.time()
    if not args.no_parity:
        dig = B.digests()
        for j in range(args.matrices):
            u = j // reps
            bad_dig += (dig[2 * j] != lb.mats[u].digest[0]) or (dig[2 * j + 1] != lb.mats[u].digest[1])
            bad_sum += B.matrix_summary_fnv(j) != lb.mats[u].summary_fnv
    t_par = time.time() - t_par
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
    traffic, traffic_info = None, None
    if args.traffic == "auto" and os.environ.get("MTB_IN_PMC") != "1":
        traffic, traffic_info = _traffic(args)
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
                     "unit": "GB/s", "frac": round(alg / (km * 1e-3) / 1e9 / HBM_PEAK_GBPS, 6), "traffic": traffic,
                     "kernel": "mtb_matrix_kernel", "kernel_ms": round(km, 3), "alg_bytes_per_launch": alg},
        "cpu_baseline": cpu,
        "parity": None if args.no_parity else {
            "matrices": args.matrices, "digest_mismatches": bad_dig, "summary_mismatches": bad_sum,
            "seconds": round(t_par, 2),
            "what": "every matrix: both vectors' GPU state digests vs the oracle's, and the FNV-1a of its SharedMatrix "
                    "summary blobs (rows / cols / handle tables / cells) vs the oracle's summary of the same log"},
        "traffic_pmc": traffic_info,
        "timing": {"generate_s": round(t_gen, 2), "load_and_first_replay_s": round(t_load, 2)},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
