#!/bin/bash
# Round 4: the SnapshotV1 serializer writing chunks and the summary directly: the GPU tests that compare summaries
# with the oracle, then the default bench (every document's SnapshotV1 fingerprint vs the oracle) with phase times.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-sumfast}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_edge_cases.py tests/test_gpu_incr.py tests/test_gpu_load.py tests/test_gpu_local.py tests/test_gpu_matrix.py tests/test_gpu_parity.py tests/test_gpu_relpos.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_summaries.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_summaries.log; [ $rc -ne 0 ] && exit $rc
export MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1 MTB_TIMING=1
timeout -k 10 600 python3 bench.py --no-cpu --steps 1 --warmup 0 --traffic off > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc $(python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['snapshot_v1'])" 2>/dev/null)"; grep mtb_timing $O/bench.err | tail -2; exit $rc
