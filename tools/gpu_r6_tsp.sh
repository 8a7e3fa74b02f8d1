# r6: K9t sample-pass period A/B (every 16th block = product vs 32nd / 64th), kernel trace
# per variant, then the threshold-scan tests on each variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base tsp32 tsp64; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/tools/abvar/$v.so; fi
  MQ_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tsp_$v -o run -- python3 -u tools/thresh_bench.py --iters 30 > gpurun_out/tsp_$v.log 2>&1 || exit 1
done
for v in tsp32 tsp64; do
  MQ_LIB_PATH=$PWD/tools/abvar/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_thresh.py > gpurun_out/tsp_${v}_tests.log 2>&1 || exit 1
done
