#!/bin/bash
# final round-4 library, part 1: C3 / C3F profile passes (stats + PMC incl. VMEM instruction counts), the bench line
set -u
mkdir -p gpurun_out
TAG=${TAG:-r04x} CONFIGS="C3 C3F" bash tools/profile_r04.sh || exit $?
