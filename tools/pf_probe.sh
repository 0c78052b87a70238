set -u
mkdir -p gpurun_out
timeout -k 10 200 python3 bench.py --per-frame-only --steps 2 --coalesce 32 > gpurun_out/pf_a.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 8 --no-cpu-baseline --no-framed > gpurun_out/pf_b.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 8 --no-cpu-baseline > gpurun_out/pf_c.log 2>&1 || exit $?
