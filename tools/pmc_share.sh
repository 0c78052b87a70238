set -e
G="TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES"
TAG=n1 ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-counters" bash tools/pmc.sh "$G"
TAG=n2 ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-counters --emulate-ranks 2" bash tools/pmc.sh "$G"
TAG=n2s1 ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-counters --emulate-ranks 2 --frame-split 1" bash tools/pmc.sh "$G"
TAG=n1s6 ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-counters --frame-split 6" bash tools/pmc.sh "$G"
