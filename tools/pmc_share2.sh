set -e
G="TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
TAG=a1s2 ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-counters --frame-split 2" bash tools/pmc.sh "$G"
TAG=a8 ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-counters --emulate-ranks 8 --frames-per-step 8" bash tools/pmc.sh "$G"
