#!/bin/bash
# Round 4: slice capacities after removing the redundant 2x re-layout: cfg4 (the long document's text slice),
# the 50,000-document shard (cfg3 at N = 2) that ran out of memory before, annotate-heavy (aux slices), and
# the -m gpu suite.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-mem}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 bench.py --workload long-doc --no-cpu --no-summary --traffic off > $O/long_doc.json 2> $O/long_doc.err
rc=$?; echo "long-doc rc=$rc $(python3 -c "import json;d=json.load(open('$O/long_doc.json'));print(d['value'],d['parity'],d['timing'])" 2>/dev/null)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --workload annotate-heavy --no-cpu --no-summary --traffic off > $O/annotate_heavy.json 2> $O/annotate_heavy.err
rc=$?; echo "annotate-heavy rc=$rc $(python3 -c "import json;d=json.load(open('$O/annotate_heavy.json'));print(d['value'],d['parity'],d['timing'])" 2>/dev/null)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 bench.py --docs-per-gpu 50000 --no-cpu --traffic off --steps 3 --warmup 1 > $O/shard_50000.json 2> $O/shard_50000.err
rc=$?; echo "50k rc=$rc $(python3 -c "import json;d=json.load(open('$O/shard_50000.json'));print(d['value'],d['parity'],d['timing'])" 2>/dev/null)"; exit $rc
