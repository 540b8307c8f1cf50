#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_v2b.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_v2b.log; if [ $rc -ne 0 ]; then exit $rc; fi
export MTB_NO_TORCH=1
B="bench.py --no-cpu --steps 1 --warmup 0 --parity-sample 4"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o trace -- python3 $B > gpurun_out/prof/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o fetch -- python3 $B > gpurun_out/prof/fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o write -- python3 $B > gpurun_out/prof/write.log 2>&1
rc=$?; echo "write rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof/sq -o sq -- python3 $B > gpurun_out/prof/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; exit $rc
