#!/bin/bash
# Per-phase device cycles (MTB_PROFILE builds) and SQ instruction counts of the observer replay on cfg2.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-prof}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_local.py tests/test_gpu_legacy.py -k "summar or parity or legacy" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
MTB_TIMING=1 timeout -k 10 600 python3 bench.py --no-cpu --steps 3 --warmup 1 --traffic off > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-300 $O/bench.json; [ $rc -ne 0 ] && exit $rc
for v in prof profpack; do
  MTB_LIB=fluidframework_amd/libmtb_$v.so MTB_PROFILE_OUT=1 timeout -k 10 600 python3 $B > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?; echo "$v rc=$rc"; grep mtb_profile $O/bench_$v.err; [ $rc -ne 0 ] && exit $rc
done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/sq -o sq -- python3 $B > $O/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --output-format csv -d $O/sq2 -o sq2 -- python3 $B > $O/sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; exit $rc
