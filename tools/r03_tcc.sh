#!/bin/bash
# L2 (TCC) hit / miss and EA request counters of the replay launch, scheduled and unscheduled, on the current build.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-tcc}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off"
for s in 1 0; do
  export MTB_SCHED=$s
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/tcc_sched$s -o tcc -- python3 $B > $O/tcc_sched$s.log 2>&1
  rc=$?; echo "tcc sched=$s rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
