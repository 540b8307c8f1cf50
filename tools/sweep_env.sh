#!/bin/bash
# Same-box sweep of an engine environment variable on the default workload (gpurun): two rounds over the
# values, ops/s and kernel time of each run, every document's digest checked.
# usage: bash tools/sweep_env.sh OUTDIR VAR VALUE [VALUE ...]   ("-" = unset)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}; VAR=${2:?var}; shift 2
mkdir -p $O
export MTB_NO_TORCH=1 MTB_LOG_CACHE=/tmp/mtb_logs TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for r in 1 2; do
  i=0
  for val in "$@"; do
    v=v$i$r; i=$((i+1))
    if [ "$val" = - ]; then unset $VAR; else export $VAR="$val"; fi
    timeout -k 10 600 python3 -u bench.py --no-cpu --no-summary --traffic off > $O/$v.json 2> $O/$v.err
    rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -3 $O/$v.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', '$VAR=$val', round(d['value']/1e6,2), 'M ops/s', d['roofline']['kernel_ms'], 'ms', 'mismatches', d['parity']['mismatches'])"
  done
  unset $VAR
done
