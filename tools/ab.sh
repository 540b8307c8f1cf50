#!/bin/bash
# Same-box A/B of two engine builds on the default workload (gpurun): B A B A, kernel time and ops/s of each,
# every document's digest checked.  usage: bash tools/ab.sh OUTDIR LIB_A [LIB_B (default: the product build)]
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; A=${2:?lib}; B=${3:-fluidframework_amd/libmtb.so}
mkdir -p $O
export MTB_NO_TORCH=1 MTB_LOG_CACHE=/tmp/mtb_logs TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for r in 1 2; do
  for v in B A; do
    lib=$B; [ $v = A ] && lib=$A
    MTB_LIB=$lib timeout -k 10 600 python3 -u bench.py --no-cpu --no-summary --traffic off > $O/$v$r.json 2> $O/$v$r.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v$r rc=$rc"; tail -3 $O/$v$r.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('$O/$v$r.json')); print('$v$r', '$lib', round(d['value']/1e6,2), 'M ops/s', d['roofline']['kernel_ms'], 'ms', 'mismatches', d['parity']['mismatches'])"
  done
done
