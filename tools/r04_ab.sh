#!/bin/bash
# Same-box A/B of replay-kernel builds on the cfg2 bench: bash tools/r03_ab.sh <outdir> <lib> <lib> ... (ABAB order)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/$1; shift
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    MTB_LIB=$lib timeout -k 10 600 python3 bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off > $O/bench_${n}_$rep.json 2> $O/bench_${n}_$rep.err
    rc=$?; echo "$n rep $rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/bench_${n}_$rep.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
