#!/bin/bash
# final round-4 library, part 2: C2 / C5 profile passes and the per-frame profile
set -u
mkdir -p gpurun_out
TAG=${TAG:-r04y} CONFIGS="C2 C5" bash tools/profile_r04.sh || exit $?
TAG=${TAG:-r04y} bash tools/profile_perframe.sh || exit $?
