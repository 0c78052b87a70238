#!/bin/bash
# PMC passes of C3 on the SAH hierarchy (the fast_bvh leg's own roofline), then the bench line that reads them
set -u
mkdir -p gpurun_out
TAG=r04x_sah CONFIGS="C3" BENCH_EXTRA="--bvh sah" bash tools/profile_r04.sh || exit $?
