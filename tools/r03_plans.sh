#!/bin/bash
# Same-box sweep of ticket chunk plans (MTB_CHUNK_PLAN) on the cfg2 bench, ABAB order.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-plans}; shift
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for rep in 1 2; do
  i=0
  for plan in "$@"; do
    i=$((i+1))
    MTB_CHUNK_PLAN=$plan timeout -k 10 600 python3 bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off > $O/bench_p${i}_$rep.json 2> $O/bench_p${i}_$rep.err
    rc=$?; echo "plan $plan rep $rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/bench_p${i}_$rep.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
