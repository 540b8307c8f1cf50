#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats of one bench step, SQ counters (separate pass).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp MTB_NO_TORCH=1
B="bench.py --no-cpu --steps 1 --warmup 0 --parity-sample 4 --traffic off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o trace -- python3 $B > gpurun_out/prof/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 gpurun_out/prof/trace.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/prof/sq -o sq -- python3 $B > gpurun_out/prof/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --output-format csv -d gpurun_out/prof/sq2 -o sq2 -- python3 $B > gpurun_out/prof/sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; exit $rc
