#!/bin/bash
# Round 4: same-box A/B of the SnapshotV1 download in pieces (MTB_SUMMARY_PIECES 1 / 8 / 32), default bench shape.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-pieces}
mkdir -p $O
export TMPDIR=/tmp MTB_LOG_CACHE=/tmp/mtb_logs MTB_NO_TORCH=1 MTB_TIMING=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for rep in 1 2; do
  for P in 1 8 32; do
    MTB_SUMMARY_PIECES=$P timeout -k 10 600 python3 bench.py --no-cpu --steps 1 --warmup 0 --traffic off > $O/p${P}_$rep.json 2> $O/p${P}_$rep.err
    rc=$?; echo "pieces $P rep $rep rc=$rc $(python3 -c "import json;d=json.load(open('$O/p${P}_$rep.json'));print(d['snapshot_v1']['seconds'],d['snapshot_v1']['mismatches'])" 2>/dev/null) $(grep extract $O/p${P}_$rep.err | tail -1)"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
