#!/bin/bash
# BASELINE configs[2] shards on one GPU: the per-GPU share of sharedstring-100k at
# N = 8 (12,500 documents), N = 4 (25,000) and N = 2 (50,000): ops/s, device memory, parity.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04/${1:-cfg3}
mkdir -p $O
export TMPDIR=/tmp
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
for n in 12500 25000 50000; do
  timeout -k 10 900 python3 bench.py --docs-per-gpu $n --no-cpu --traffic off --steps 3 --warmup 1 > $O/shard_$n.json 2> $O/shard_$n.err
  rc=$?; echo "docs $n rc=$rc"; cut -c1-300 $O/shard_$n.json; [ $rc -ne 0 ] && exit $rc
done
exit 0
