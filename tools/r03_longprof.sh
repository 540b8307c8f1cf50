#!/bin/bash
# Per-phase device cycles of the cfg4 long document (one wave, mtb_replay_few_kernel) from an MTB_PROFILE build.
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03/${1:-longprof}
mkdir -p $O
export TMPDIR=/tmp MTB_NO_TORCH=1
(while sleep 50; do echo "hb $(date +%T)" >> $O/heartbeat; done) & HB=$!
trap "kill $HB" EXIT
MTB_LIB=fluidframework_amd/libmtb_prof.so MTB_PROFILE_OUT=1 timeout -k 10 1000 python3 -u bench.py --workload long-doc --no-cpu --no-summary --traffic off > $O/long_prof.json 2> $O/long_prof.err
rc=$?; echo "long prof rc=$rc"; grep mtb_profile $O/long_prof.err; cut -c1-200 $O/long_prof.json; exit $rc
