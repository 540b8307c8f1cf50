#!/bin/bash
# Round 4: host phase times (MTB_TIMING=1) of the SnapshotV1 leg of the default bench: extraction on the GPU +
# download vs host serialization, at 16 and 8 summary threads.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-sumtime}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1 MTB_TIMING=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for t in 16 8; do
  timeout -k 10 600 python3 bench.py --no-cpu --steps 1 --warmup 0 --traffic off --summary-threads $t > $O/bench_t$t.json 2> $O/bench_t$t.err
  rc=$?; echo "t=$t rc=$rc"; grep "mtb_timing" $O/bench_t$t.err | tail -3; [ $rc -ne 0 ] && exit $rc
done
exit 0
