# Short N=1 bench of the in-tree library and of variants/*.so builds (A/B of a kernel change).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --single-iters 20 > gpurun_out/bv_main.json 2>/dev/null || { echo MAIN_FAIL; exit 1; }
for v in variants/*.so; do
  n=$(basename $v .so)
  MQ_LIB_PATH=$PWD/$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --single-iters 20 > gpurun_out/bv_$n.json 2>/dev/null || { echo FAIL $n; exit 1; }
done
echo BV_OK
