#!/bin/bash
# GPU: matrix / load parity tests (PermutationVector body chunks), then PC sampling of the replay kernel.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-next}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_matrix.py tests/test_gpu_load.py tests/test_gpu_local.py -k "matrix or load or summaries" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/r03_pcs.sh ${1:-next}
