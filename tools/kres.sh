#!/bin/bash
# Per-kernel resource usage (VGPRs, spills, occupancy) of the replay engine: tools/kres.sh [extra hipcc flags]
cd /tmp && hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c /root/repo/fluidframework_amd/csrc/mtb_replay.hip -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | python3 -c '
import sys,re
cur=None
for l in sys.stdin:
    m=re.search(r"remark: +(Function Name|VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)",l)
    if not m: continue
    k,v=m.groups()
    if k=="Function Name": cur=v; print(); print(v.ljust(26),end="")
    else: print(" %s=%s"%(k.split()[0] if "Spill" not in k else k.replace(" ",""),v),end="")
print()'
