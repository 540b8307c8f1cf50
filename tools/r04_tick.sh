#!/bin/bash
# Round 4: one ticket per workgroup (mtb_replay_tick_kernel: the plain engine's register allocation, no scratch)
# as the scheduled replay: cfg2 for the default chunk plan (twice) and 16 equal chunks, the -m gpu suite without
# the persistent-ticket cases, then the matrix bench (total parity incl. summaries).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-tick}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off"
for v in plan_1 c16 plan_2; do
  if [ $v = c16 ]; then export MTB_CHUNKS=16; else unset MTB_CHUNKS; fi
  timeout -k 10 600 python3 $B > $O/tick_$v.json 2> $O/tick_$v.err
  rc=$?; echo "$v rc=$rc $(python3 -c "import json;d=json.load(open('$O/tick_$v.json'));print(d['value'],d['roofline']['kernel_ms'],d['roofline']['launch'],d['parity']['mismatches'])" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
unset MTB_CHUNKS
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not tickets" > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 bench_matrix.py > $O/matrix.json 2> $O/matrix.err
rc=$?; echo "matrix rc=$rc"; cut -c1-700 $O/matrix.json; exit $rc
