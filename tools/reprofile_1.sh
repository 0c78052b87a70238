#!/bin/bash
# After a library change, part 1 (tools/reprofile_after_library_change.md): C3 / C3F profile passes (stats + PMC), then the per-frame profile (server on / off)
set -u
mkdir -p gpurun_out
TAG=${TAG:?set TAG} CONFIGS="C3 C3F" bash tools/profile_r04.sh || exit $?
TAG=${TAG:?set TAG} bash tools/profile_perframe.sh || exit $?
