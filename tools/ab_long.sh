#!/bin/bash
# Same-box comparison of engine builds on cfg4 (bench.py --workload long-doc: one 1M-char document, 1M ops):
# two rounds over the product build and each variant, ops/s and digest of each run.
# usage: bash tools/ab_long.sh OUTDIR LIB [LIB ...]
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; shift
mkdir -p $O
export MTB_NO_TORCH=1 MTB_LOG_CACHE=/tmp/mtb_logs TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for r in 1 2; do
  i=0
  for lib in fluidframework_amd/libmtb.so "$@"; do
    v=v$i$r; i=$((i+1))
    MTB_LIB=$lib timeout -k 10 600 python3 -u bench.py --workload long-doc --no-cpu --no-summary --traffic off --parity-sample 1 > $O/$v.json 2> $O/$v.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -3 $O/$v.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', '$lib', round(d['value']), 'ops/s', d['roofline']['kernel_ms'], 'ms', 'mismatches', d['parity']['mismatches'])"
  done
done
