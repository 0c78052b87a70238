#!/bin/bash
# Compact resource report of the timed regen/stream kernels: make resource with EXTRA="$*"
make -s -C "$(dirname "$0")/../halogen-pathtracer_amd" resource KERNEL=hg_mega EXTRA="$*" 2>&1 |
  python3 -c "
import re,sys
cur=None
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); print(); print(cur[:45],end=' ')
    for k in ('VGPRs:','SGPRs Spill:','VGPRs Spill:','ScratchSize \[bytes/lane\]:','Occupancy \[waves/SIMD\]:'):
        m=re.search(k+r' (\d+)',l)
        if m: print(k.split()[0].replace('\\\\',''),m.group(1),end=' ')
print()" | grep -E 'ILb0E'
