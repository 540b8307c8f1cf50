#!/bin/bash
# GPU tests of marker ids (reused ids, assert 0x5ad) and the relative-position / load suites they touch.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-mk}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_relpos.py tests/test_gpu_load.py tests/test_gpu_edge_cases.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $O/pytest.log; exit $rc
