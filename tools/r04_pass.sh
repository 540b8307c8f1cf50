#!/bin/bash
# Round 4: replay in passes (mtb_replay_pass_kernel, the plain engine's code generation, no scratch) instead
# of the ticket-scheduled persistent kernel: cfg2 bench for the chosen chunk count and for 4 and 6 chunks per
# document, then the -m gpu suite without the ticket-kernel tests.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-pass}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
B="bench.py --no-cpu --no-summary --steps 3 --warmup 1 --traffic off"
for m in default 4 6 default; do
  if [ $m = default ]; then unset MTB_PASS_CHUNKS; else export MTB_PASS_CHUNKS=$m; fi
  timeout -k 10 600 python3 $B > $O/pass_$m.json 2> $O/pass_$m.err
  rc=$?; echo "chunks $m rc=$rc $(python3 -c "import json;d=json.load(open('$O/pass_$m.json'));print(d['value'],d['roofline']['kernel_ms'],d['roofline']['launch'],d['parity']['mismatches'])" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
unset MTB_PASS_CHUNKS
for lib in libmtb_rbl libmtb_rbd libmtb_rbx; do  # rebuild() variants (same-box A/B against pass_default)
  MTB_LIB=fluidframework_amd/$lib.so timeout -k 10 600 python3 $B > $O/ab_$lib.json 2> $O/ab_$lib.err
  rc=$?; echo "$lib rc=$rc $(python3 -c "import json;d=json.load(open('$O/ab_$lib.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])" 2>/dev/null)"
  [ $rc -ne 0 ] && exit $rc
done
for v in prof profpack; do  # per-phase cycle counters (MTB_PROFILE builds)
  MTB_LIB=fluidframework_amd/libmtb_$v.so MTB_PROFILE_OUT=1 timeout -k 10 600 python3 bench.py --no-cpu --no-summary --steps 1 --warmup 0 --parity-sample 4 --traffic off > $O/bench_$v.json 2> $O/bench_$v.err
  rc=$?; echo "$v rc=$rc"; grep "mtb_profile" $O/bench_$v.err; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "not scheduled_replay" > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; exit $rc
