#!/bin/bash
# Round-3 baseline on the GPU box: default bench (driver command), then L2 hit/miss counters of the replay
# launch with and without ticket scheduling (is the L2 write-back/invalidate the cause?).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-base}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err.log
rc=$?; echo "bench rc=$rc"; cat $O/bench.json; [ $rc -ne 0 ] && exit $rc
B="bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off"
export MTB_NO_TORCH=1
for s in 1 0; do
  export MTB_SCHED=$s
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/tcc_sched$s -o tcc -- python3 $B > $O/tcc_sched$s.log 2>&1
  rc=$?; echo "tcc sched=$s rc=$rc"; tail -1 $O/tcc_sched$s.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
