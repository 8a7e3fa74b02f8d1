# A/B one environment knob on the N=1 bench: BENV="VAR=value" bash tools/ab_env.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --single-iters 20 > gpurun_out/ab_a.json 2>/dev/null || { echo A_FAIL; exit 1; }
env $BENV timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --single-iters 20 > gpurun_out/ab_b.json 2>/dev/null || { echo B_FAIL; exit 1; }
echo AB_OK
