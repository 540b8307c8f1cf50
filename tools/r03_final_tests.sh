#!/bin/bash
# Round-end GPU evidence, part 1: the whole `pytest -m gpu` suite and __graft_entry__.smoke() on the committed build.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; exit $rc
