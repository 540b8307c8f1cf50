"""Benchmark of SURVEY.md 8(f) rank 1: SnapshotV1 summary load (Client.load -> SnapshotLoader).

Workload: the headline workload's documents (8 writer clients x 10,000 messages, insert/remove/annotate
50/30/20%), each summarized by the engine at quiescence (updateSeqNumbers(seq, seq): every segment at
or below the MSN) with mergeTreeSnapshotChunkSize = --chunk (so most segments travel in body chunks).
One step = load every summary into a fresh batch of --docs documents: the host parses the blobs on
--threads threads (mtb_docs_load_v1) and rebuilds each header as a device tree (reloadFromSegments + startCollaboration), uploads it, and the
loader kernel appends every body chunk on the GPU (insertSegments of NonCollab segments at the end of
the document).  The blobs are host buffers (the reference reads them from storage), so the timed region
includes host parsing and PCIe upload; the loader kernel's own time is reported beside it.

value = summary segments loaded per second, whole step.  The roofline line is for mtb_load_kernel:
algorithmic bytes per body segment = its 32-byte record + its text (2 B/unit) + the 24-byte segment
written into its block record.

cpu_baseline: the C++ oracle's restatement of SnapshotLoader (oracle/, kind "port") loading a bounded
sample of the same summaries on one host core.
"""
import argparse
import ctypes
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
    ap.add_argument("--docs", type=int, default=10000)
    ap.add_argument("--replicas", type=int, default=10)
    ap.add_argument("--ops", type=int, default=10000)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=1000, help="mergeTreeSnapshotChunkSize of the summarizer")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=300)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=20260202)
    ap.add_argument("--threads", type=int, default=16, help="host threads parsing summaries (mtb_docs_load_v1)")
    args = ap.parse_args()

    from fluidframework_amd import MergeTreeBatch, _lib
    from pyloggen import LogBatch, make_cfg

    reps = max(1, args.replicas)
    n_unique = (args.docs + reps - 1) // reps
    cfg = make_cfg(seed=args.seed, n_clients=args.clients, n_ops=args.ops)
    t0 = time.time()
    lb = LogBatch(cfg, 0, n_unique, threads=min(16, os.cpu_count() or 1))
    # summaries: replay every log on the GPU and summarize at quiescence
    A = MergeTreeBatch(n_unique, chunk_size=args.chunk)
    for p in lb.props_json()[1:]:
        A.intern_props(p)
    for u in range(n_unique):
        d = lb.docs[u]
        tb = lb.doc_text_bytes(u)
        A.init_doc(u, tb[: d.initial_len * 2].decode("utf-16-le"), "obs")
        for cid in lb.client_ids(u)[1:]:
            A.add_client(u, cid)
        A.append_records(u, lb.doc_ops_bytes(u), d.n_ops, tb)
    st = A.replay()
    if st["errors"]:
        raise SystemExit("summary source replay failed")
    summaries, texts = [], []
    body_segs = body_units = all_segs = 0
    for u in range(n_unique):
        seq = A.seq(u)[0]
        blobs, _ = A.summarize_v1(u, seq, seq)
        summaries.append(blobs)
        texts.append(A.text(u))
        for path, content in blobs:
            segs = json.loads(content)["segments"]
            all_segs += len(segs)
            if path != "header":
                body_segs += len(segs)
                body_units += sum(len(s) if isinstance(s, str) else (len(s["text"]) if "text" in s else 0) for s in segs)
    t_prep = time.time() - t0
    # host blob arrays for the ABI (built once, outside the timed region)
    keep, arrays = [], []
    ap_threads = args.threads
    for blobs in summaries:
        arr = (_lib.MtbBlob * len(blobs))()
        for i, (p, c) in enumerate(blobs):
            pb, cb = p.encode(), c.encode()
            buf = ctypes.create_string_buffer(cb, len(cb))
            keep += [pb, buf]
            arr[i].path = pb
            arr[i].content = ctypes.cast(buf, ctypes.c_void_p)
            arr[i].content_len = len(cb)
        arrays.append(arr)
    L = _lib.lib()
    docs_arr = (ctypes.c_uint32 * args.docs)(*range(args.docs))
    ptrs = (ctypes.POINTER(_lib.MtbBlob) * args.docs)(
        *[ctypes.cast(arrays[j // reps], ctypes.POINTER(_lib.MtbBlob)) for j in range(args.docs)])
    counts = (ctypes.c_uint32 * args.docs)(*[len(summaries[j // reps]) for j in range(args.docs)])
    obs = (ctypes.c_char_p * args.docs)(*([b"obs"] * args.docs))

    def step():
        B = MergeTreeBatch(args.docs, chunk_size=args.chunk)
        th = time.perf_counter()
        B._chk(L.mtb_docs_load_v1(B._h, args.docs, docs_arr, ptrs, counts, obs, ap_threads))
        B._dirty = True
        host = time.perf_counter() - th
        s = B.replay()
        return B, host, s

    for _ in range(args.warmup):
        step()
    times, hosts, kms = [], [], []
    B = None
    for _ in range(args.steps):
        t0 = time.perf_counter()
        B, host, s = step()
        times.append(time.perf_counter() - t0)
        hosts.append(host)
        kms.append(s["kernel_ms"])
        if s["errors"]:
            raise SystemExit("load errors")
    # parity sample: text equals the source document's; the loaded document summarizes back to the same bytes
    bad = 0
    sample = list(range(0, args.docs, max(1, args.docs // 32)))[:32]
    for j in sample:
        u = j // reps
        seq = A.seq(u)[0]
        if B.text(j) != texts[u] or [tuple(x) for x in B.summarize_v1(j, seq, seq)[0]] != [tuple(x) for x in summaries[u]]:
            bad += 1

    el = sum(times) / len(times)
    km = sum(kms) / len(kms)
    segs_step = all_segs * args.docs / n_unique
    body_step = body_segs * args.docs / n_unique
    units_step = body_units * args.docs / n_unique
    alg = 32 * body_step + 2 * units_step + 24 * body_step
    cpu = None
    if not args.no_cpu:
        from pyoracle import OracleDoc
        k = min(args.cpu_sample, n_unique)
        segs = 0
        t0 = time.perf_counter()
        for u in range(k):
            o = OracleDoc()
            o.load_v1(summaries[u], "obs")
            o.close()
        secs = time.perf_counter() - t0
        for u in range(k):
            segs += sum(len(json.loads(c)["segments"]) for _, c in summaries[u])
        cpu = {"value": round(segs / secs, 1), "unit": "segments/s", "cores": 1, "kind": "port",
               "sample": f"{k} of the same summaries ({segs} segments) loaded by the C++ oracle (oracle/), 1 thread, {secs:.2f}s"}
    out = {
        "metric": "SnapshotV1 summary segments loaded/sec (Client.load), 10k-doc batch",
        "value": round(segs_step / el, 1),
        "unit": "segments/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el * 1e3, 3),
        "higher_is_better": True,
        "dtype": "int32",
        "data": f"synthetic: {n_unique} generated logs summarized at quiescence, each loaded as {reps} documents",
        "config": {"workload": f"summary-load: {args.docs} docs, {args.clients} clients x {args.ops} msgs each, "
                               f"chunk size {args.chunk}, {ap_threads} host parse threads", "segments_per_step": int(segs_step),
                   "body_segments_per_step": int(body_step)},
        "roofline": {"bound": "hbm", "achieved": round(alg / (km * 1e-3) / 1e9, 3), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(alg / (km * 1e-3) / 1e9 / HBM_PEAK_GBPS, 6), "traffic": None,
                     "kernel": "mtb_load_kernel (+ an empty mtb_replay_kernel pass)", "kernel_ms": round(km, 3),
                     "alg_bytes_per_launch": int(alg)},
        "cpu_baseline": cpu,
        "parity": {"sampled_docs": len(sample), "mismatches": bad},
        "timing": {"host_parse_and_tree_build_ms": round(sum(hosts) / len(hosts) * 1e3, 1),
                   "flush_ms": round((el - sum(hosts) / len(hosts)) * 1e3, 1), "prep_s": round(t_prep, 1)},
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
