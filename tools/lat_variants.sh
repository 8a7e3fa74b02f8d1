# Single-query latency of the in-tree library and of variants/*.so builds (A/B of build knobs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/lat_main.json 2>&1 || { echo MAIN_FAIL; exit 1; }
for v in variants/*.so; do
  n=$(basename $v .so)
  MQ_LIB_PATH=$PWD/$v timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/lat_$n.json 2>&1 || { echo FAIL $n; exit 1; }
done
echo LAT_OK
