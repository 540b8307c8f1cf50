#!/bin/bash
# PC sampling (host trap) of the scheduled replay kernel on a reduced cfg2-shaped run (5,000 docs x 3,000 msgs).
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-pcs}
mkdir -p $O
export TMPDIR=/tmp MTB_NO_TORCH=1 MTB_LIB=fluidframework_amd/libmtb_g.so
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --output-format csv -d $O/pcs -o pcs -- python3 bench.py --no-cpu --no-summary --steps 1 --warmup 0 --traffic off --docs-per-gpu 5000 --ops 3000 > $O/pcs.log 2>&1
rc=$?; echo "pcs rc=$rc"; tail -3 $O/pcs.log; find $O/pcs -name "*.csv" | head; exit $rc
