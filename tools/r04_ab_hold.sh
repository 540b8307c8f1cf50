#!/bin/bash
# Round 4: same-box A/B of packParent's list rebuild from hold[] (libmtb_hold.so) against the tick-kernel
# baseline (libmtb.so), both with the 12,3,1 ticket plan, ABAB; then the cfg3 shards (tools/r04_cfg3.sh).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-ab_hold}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off"
for rep in 1 2; do
  for lib in libmtb libmtb_hold; do
    MTB_LIB=fluidframework_amd/$lib.so timeout -k 10 600 python3 $B > $O/${lib}_$rep.json 2> $O/${lib}_$rep.err
    rc=$?; echo "$lib rep $rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/${lib}_$rep.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
unset MTB_NO_TORCH MTB_LOG_CACHE
bash tools/r04_cfg3.sh ${1:-ab_hold}/cfg3
