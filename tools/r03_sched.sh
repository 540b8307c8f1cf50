#!/bin/bash
# Scheduler v2 check: scheduled-replay parity tests (queues, forced abort), then bench A/B of per-XCD queues
# vs one global queue, with L2 counters of each.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-sched}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_local.py tests/test_gpu_matrix.py -k "scheduled or divergence or conflict_kats" > $O/pytest_sched.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_sched.log; [ $rc -ne 0 ] && exit $rc
B="bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off"
for q in 8 1; do
  MTB_SCHED_QUEUES=$q timeout -k 10 600 python3 $B > $O/bench_q$q.json 2> $O/bench_q$q.err
  rc=$?; echo "bench q=$q rc=$rc"; cut -c1-400 $O/bench_q$q.json; [ $rc -ne 0 ] && exit $rc
done
export MTB_NO_TORCH=1
for q in 8 1; do
  export MTB_SCHED_QUEUES=$q
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/tcc_q$q -o tcc -- python3 bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off > $O/tcc_q$q.log 2>&1
  rc=$?; echo "tcc q=$q rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
