"""bench.py's multi-rank path on one GPU (MTB_BENCH_SHARE_GPU=1: every rank on device 0, counters reduced
over gloo instead of RCCL): torchrun with two ranks replays BASELINE configs[2]'s workload shape (documents in
total sharded by hash(doc) mod N, "scaling": "strong") with a small document count, and the one JSON line of
rank 0 reports every document's digest parity and SnapshotV1 fingerprints over both ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_share_one_gpu():
    env = dict(os.environ, MTB_BENCH_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("MTB_NO_TORCH", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--docs-total", "300", "--ops", "600", "--traffic", "off"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["config"]["docs_total"] == 300 and out["config"]["workload"].startswith("sharedstring-100k")
    assert out["parity"]["sampled_docs"] == 300 and out["parity"]["mismatches"] == 0 and out["parity"]["errors"] == 0
    assert out["snapshot_v1"]["documents"] == 300 and out["snapshot_v1"]["mismatches"] == 0
    assert out["cpu_baseline"] is None  # (an N = 1 figure)
    assert out["value"] > 0


def test_bench_gpus_2_without_launcher():
    """`python bench.py --gpus 2` with no torchrun: bench.py starts its two ranks itself (under
    torch.distributed.run, before any GPU call) and reports n_gpus == 2 with every document checked."""
    env = dict(os.environ, MTB_BENCH_SHARE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("MTB_NO_TORCH", "WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--docs-total", "300", "--ops", "600", "--traffic", "off"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong"
    assert out["parity"]["sampled_docs"] == 300 and out["parity"]["mismatches"] == 0 and out["parity"]["errors"] == 0
    assert out["snapshot_v1"]["documents"] == 300 and out["snapshot_v1"]["mismatches"] == 0
    assert out["timing"]["generator_threads_per_rank"] >= 1
