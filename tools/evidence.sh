#!/bin/bash
# Round-end GPU evidence on the current build (run through gpurun): the default bench line (CPU baseline, PMC
# traffic passes, SnapshotV1 at scale), a rocprofv3 kernel trace + stats of one bench step, SQ and TCC counter
# passes (one counter set per run), the MTB_PROFILE phase counters (tools/build_variants.py prof, profpack),
# then cfg4 (the long document) with its own SQ passes and phase counters.
# usage: bash tools/evidence.sh OUTDIR [long]   (OUTDIR under gpurun_out/; "long": only the cfg4 part)
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:?outdir}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
exec 3>&1  # (step's status line goes to the call's stdout, not into a step's redirected output)
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >&3; [ $rc -ne 0 ] && exit $rc; return 0; }
if [ "$2" != long ]; then
step bench timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err.log
cut -c1-300 $O/bench.json
export MTB_NO_TORCH=1 MTB_LOG_CACHE=/tmp/mtb_logs
B="bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off"
step trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $B > $O/trace.log 2>&1
step sq timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/sq -o sq -- python3 $B > $O/sq.log 2>&1
step sq2 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --output-format csv -d $O/sq2 -o sq2 -- python3 $B > $O/sq2.log 2>&1
step tcc timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/tcc -o tcc -- python3 $B > $O/tcc.log 2>&1
for v in prof; do  # (the MTB_PROFILE_PACK build faulted in round 5: DESIGN.md section 4, not run)
  step $v env MTB_LIB=tools/lib/libmtb_$v.so MTB_PROFILE_OUT=1 timeout -k 10 600 python3 $B > $O/bench_$v.json 2> $O/bench_$v.err
  grep "mtb_profile" $O/bench_$v.err
done
fi
export MTB_NO_TORCH=1
L="bench.py --workload long-doc --steps 1 --warmup 0 --traffic off --no-summary"
step long_doc timeout -k 10 600 python3 -u $L > $O/long_doc.json 2> $O/long_doc.err
cut -c1-300 $O/long_doc.json
LP="$L --no-cpu --parity-sample 1"
step long_sq timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O/long_sq -o sq -- python3 $LP > $O/long_sq.log 2>&1
step long_sq2 timeout -s KILL 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM --output-format csv -d $O/long_sq2 -o sq2 -- python3 $LP > $O/long_sq2.log 2>&1
step long_prof env MTB_LIB=tools/lib/libmtb_prof.so MTB_PROFILE_OUT=1 timeout -k 10 600 python3 -u $LP > $O/long_prof.json 2> $O/long_prof.err
grep mtb_profile $O/long_prof.err
