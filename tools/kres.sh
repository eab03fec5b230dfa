#!/bin/bash
# Print per-kernel resource usage (VGPR, SGPR, scratch, LDS, occupancy) of a HIP source.
src=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
  -I/root/repo/include -I/root/repo/orbslam2commentedbyxcm_amd/csrc -c "$src" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | python3 -c '
import sys,re
cur=None
for line in sys.stdin:
    m=re.search(r"Function Name: (\S+)",line)
    if m: cur=m.group(1); print(); print(cur[:60].ljust(60),end=""); continue
    for k in ["VGPRs:","ScratchSize \[bytes/lane\]:","Occupancy \[waves/SIMD\]:","LDS Size \[bytes/block\]:","TotalSGPRs:"]:
        m=re.search(k+r" (\d+)",line)
        if m: print(" %s=%s"%(k.split()[0].strip(":"),m.group(1)),end="")
print()'
