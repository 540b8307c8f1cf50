#!/bin/bash
# Round 4: the whole -m gpu suite, the packParent profile builds (MTB_CHECK bounds-checked MTB_PROFILE_PACK,
# MTB_PROFILE_PACK, MTB_PROFILE) on cfg2, a same-box A/B of the rebuild variants, then the matrix bench.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-second}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off"
for v in check profpack prof; do
  MTB_LIB=fluidframework_amd/libmtb_$v.so MTB_PROFILE_OUT=1 MTB_CHECK_OUT=1 timeout -k 10 600 python3 $B > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?; echo "$v rc=$rc"; grep "mtb_profile\|mtb_check" $O/bench_$v.err; [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2; do
  for lib in fluidframework_amd/libmtb.so fluidframework_amd/libmtb_rbl.so fluidframework_amd/libmtb_rbd.so fluidframework_amd/libmtb_rbx.so; do
    n=$(basename $lib .so)
    MTB_LIB=$lib timeout -k 10 600 python3 bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off > $O/ab_${n}_$rep.json 2> $O/ab_${n}_$rep.err
    rc=$?; echo "$n rep $rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/ab_${n}_$rep.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])" 2>/dev/null)"
    [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 bench_matrix.py > $O/matrix.json 2> $O/matrix.err
rc=$?; echo "matrix rc=$rc"; cut -c1-600 $O/matrix.json; exit $rc
