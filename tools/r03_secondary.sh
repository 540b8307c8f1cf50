#!/bin/bash
# Secondary workloads on the current kernel: cfg2 in the new length calculation,
# annotate-heavy (cfg5 SharedString half), SharedMatrix (cfg5), and the cfg4 long document.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-secondary}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.json 2> $O/$n.err
  local rc=$?; echo "$n rc=$rc"; cut -c1-260 $O/$n.json; return $rc
}
run newmode 900 python3 bench.py --new-length-calc --traffic off || exit $?
run annotate_heavy 900 python3 bench.py --workload annotate-heavy --traffic off || exit $?
run matrix 900 python3 bench_matrix.py || exit $?
run long_doc 1100 python3 bench.py --workload long-doc --traffic off || exit $?
exit 0
