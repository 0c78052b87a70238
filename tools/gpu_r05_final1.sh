#!/bin/bash
# round-5 library, part 1: C3 / C3F profile passes (stats + PMC), then the per-frame profile (server on / off)
set -u
mkdir -p gpurun_out
TAG=${TAG:-r05x} CONFIGS="C3 C3F" bash tools/profile_r04.sh || exit $?
TAG=${TAG:-r05x} bash tools/profile_perframe.sh || exit $?
