#!/bin/bash
# Round 4: tick-kernel chunk plans on cfg2 (MTB_CHUNK_PLAN: relative ticket sizes per document), same box.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-plans}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off"
i=0
for plan in ${PLANS:-6,4,2,1,1,1,1 8,4,2,1,1 10,4,2 4,4,4,2,1,1 12,3,1 6,4,2,1,1,1,1}; do
  i=$((i+1))
  MTB_CHUNK_PLAN=$plan timeout -k 10 600 python3 $B > $O/plan_$i.json 2> $O/plan_$i.err
  rc=$?; echo "plan $plan rc=$rc $(python3 -c "import json;d=json.load(open('$O/plan_$i.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
