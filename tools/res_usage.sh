#!/bin/bash
# Per-kernel VGPRs / SGPRs / scratch / occupancy of hg_mega.hip as the library builds it (compare before / after a change)
cd "$(dirname "$0")/../halogen-pathtracer_amd"
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -DHG_FAST_RCP=1 -DHG_MEGA_WAVES=6 -DHG_MEGA_LDS_STACK=16 -DHG_LOCK_WAVES=4 -I../include -Icsrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 $F -c csrc/hg_mega.hip -o /tmp/res_probe.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' | awk '/Function Name/{n=$3} /VGPRs:/{v=$2} /TotalSGPRs/{sg=$2} /ScratchSize/{sc=$NF} /Occupancy/{print n, "vgpr", v, "sgpr", sg, "scratch", sc, "occ", $NF}' | grep -E "${1:-stream}"
