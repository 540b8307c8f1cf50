#!/bin/bash
# Round 4: same-box A/B of a variant library (fluidframework_amd/$2.so) against libmtb.so, ABAB on cfg2
# (3 timed steps each, all digests checked), then one cfg4 long-document run each.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-ab}
V=${2:-libmtb_heap}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off"
for rep in 1 2; do
  for lib in libmtb $V; do
    MTB_LIB=fluidframework_amd/$lib.so timeout -k 10 600 python3 $B > $O/${lib}_$rep.json 2> $O/${lib}_$rep.err
    rc=$?; echo "$lib rep $rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/${lib}_$rep.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
L="bench.py --workload long-doc --steps 1 --warmup 0 --traffic off --no-summary --no-cpu"
for lib in libmtb $V; do
  MTB_LIB=fluidframework_amd/$lib.so timeout -k 10 600 python3 -u $L > $O/long_$lib.json 2> $O/long_$lib.err
  rc=$?; echo "long $lib rc=$rc"; cut -c1-300 $O/long_$lib.json; [ $rc -ne 0 ] && exit $rc
done
exit 0
