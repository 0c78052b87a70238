#!/bin/bash
# round-3 final library: smoke + -m gpu suite + bench line, then the per-frame rocprof profile (TAG)
set -u
bash tools/gpu_r03.sh || exit $?
TAG=${TAG:-r03i} bash tools/profile_perframe.sh || exit $?
