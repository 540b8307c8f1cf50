"""bench.py's command line on the CPU: --gpus against the launcher's WORLD_SIZE, and the per-rank log
generation plan that keeps BASELINE configs[2] at N = 8 inside the driver's bench window."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _run(args, **env):
    e = dict(os.environ, **env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, cwd=ROOT,
                          capture_output=True, text=True, timeout=120)


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "3"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "--gpus 3 but the launcher started WORLD_SIZE=2" in r.stderr


def test_gpus_zero_is_rejected():
    r = _run(["--gpus", "0"])
    assert r.returncode != 0 and "must be >= 1" in r.stderr


def test_gen_plan_splits_cpus_over_ranks():
    # a 16-CPU quota shared by 8 ranks: 2 generator threads each, not 16
    assert bench.gen_plan(12500, 10000, 16, 8, 0)[0] == 2
    assert bench.gen_plan(12500, 10000, 128, 8, 0)[0] == 16
    assert bench.gen_plan(10000, 10000, 16, 1, 1) == (16, 1)  # the headline workload: every log unique
    assert bench.gen_plan(10, 10000, 16, 2, 0, gen_threads=3) == (3, 1)


def test_cfg3_generation_fits_the_bench_window():
    """configs[2] (100,000 documents x 10,000 msgs) at N = 1, 2, 4, 8 on a 16-CPU node: every rank's unique logs
    generate within the budget (estimate at the measured generator rate), far inside the 600 s window."""
    for n in (1, 2, 4, 8):
        per_rank = -(-100000 // n)
        threads, reps = bench.gen_plan(per_rank, 10000, 16, n, 0)
        unique = -(-per_rank // reps)
        gen_s = unique * 10000 / (threads * bench.GEN_MSGS_PER_THREAD_S)
        assert gen_s <= bench.GEN_BUDGET_S * 1.01, (n, threads, reps, gen_s)
        assert reps * unique >= per_rank
