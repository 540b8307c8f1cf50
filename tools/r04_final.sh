#!/bin/bash
# Round-4 GPU evidence on the current build: the default bench line (CPU baseline, PMC traffic passes,
# SnapshotV1 at scale), a rocprofv3 kernel trace + stats of one bench step, SQ and TCC counter passes (one run
# each), then cfg4 (long document) on the normal and the MTB_PROFILE build for the per-op breakdown.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err.log
rc=$?; echo "bench rc=$rc"; cut -c1-500 $O/bench.json; [ $rc -ne 0 ] && exit $rc
export MTB_NO_TORCH=1 MTB_LOG_CACHE=/tmp/mtb_logs
B="bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $B > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/sq -o sq -- python3 $B > $O/sq.log 2>&1
rc=$?; echo "sq rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --output-format csv -d $O/sq2 -o sq2 -- python3 $B > $O/sq2.log 2>&1
rc=$?; echo "sq2 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/tcc -o tcc -- python3 $B > $O/tcc.log 2>&1
rc=$?; echo "tcc rc=$rc"; [ $rc -ne 0 ] && exit $rc
for v in prof profpack; do  # per-phase cycle counters (MTB_PROFILE builds) on cfg2, tick-scheduled
  MTB_LIB=fluidframework_amd/libmtb_$v.so MTB_PROFILE_OUT=1 timeout -k 10 600 python3 $B > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?; echo "$v rc=$rc"; grep "mtb_profile" $O/bench_$v.err; [ $rc -ne 0 ] && exit $rc
done
L="bench.py --workload long-doc --steps 1 --warmup 0 --traffic off --no-summary"
timeout -k 10 600 python3 -u $L > $O/long_doc.json 2> $O/long_doc.err
rc=$?; echo "long-doc rc=$rc"; cut -c1-400 $O/long_doc.json; [ $rc -ne 0 ] && exit $rc
MTB_LIB=fluidframework_amd/libmtb_prof.so MTB_PROFILE_OUT=1 timeout -k 10 600 python3 -u $L --no-cpu > $O/long_prof.json 2> $O/long_prof.err
rc=$?; echo "long-prof rc=$rc"; grep mtb_profile $O/long_prof.err; exit $rc
