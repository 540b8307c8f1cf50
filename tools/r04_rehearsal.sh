#!/bin/bash
# Round 4, end of round: what the driver runs on a fresh box -- the -m gpu suite, smoke(), the default bench --
# on the final tree, plus the bench's host phase times (MTB_TIMING) for the SnapshotV1 leg.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-rehearsal}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
MTB_TIMING=1 timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc $(python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['parity']['mismatches'],d['snapshot_v1']['seconds'],d['snapshot_v1']['summaries_per_s'],d['snapshot_v1']['mismatches'])" 2>/dev/null)"; grep mtb_timing $O/bench.err | tail -2; exit $rc
