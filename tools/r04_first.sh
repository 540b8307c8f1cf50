#!/bin/bash
# Round 4, first GPU pass: the whole -m gpu suite on the new build, then the packParent-profile builds on cfg2:
# MTB_CHECK (slice-bounds-checked MTB_PROFILE_PACK build, reports out-of-slice accesses instead of faulting),
# then the plain MTB_PROFILE_PACK and MTB_PROFILE builds (phase breakdowns); then the matrix bench with total
# parity and PMC traffic.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-first}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
B="bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off"
for v in check profpack prof; do
  MTB_LIB=fluidframework_amd/libmtb_$v.so MTB_PROFILE_OUT=1 MTB_CHECK_OUT=1 timeout -k 10 600 python3 $B > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?; echo "$v rc=$rc"; grep "mtb_profile\|mtb_check" $O/bench_$v.err; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 900 python3 bench_matrix.py > $O/matrix.json 2> $O/matrix.err
rc=$?; echo "matrix rc=$rc"; cut -c1-400 $O/matrix.json; exit $rc
