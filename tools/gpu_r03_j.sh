#!/bin/bash
# final round-3 library: smoke + -m gpu suite + bench line, the per-frame profile and the four-config profile passes (TAG)
set -u
bash tools/gpu_r03.sh || exit $?
TAG=${TAG:-r03j} bash tools/profile_perframe.sh || exit $?
TAG=${TAG:-r03j} bash tools/profile_r03.sh || exit $?
