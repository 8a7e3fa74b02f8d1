# A/B the fp32 GEMM core: tools/base_libmqhip.so (previous build) vs the in-tree build.
# Run from the repo root on the GPU box: bash tools/ab_gemm.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 env MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$PWD/tools/base_libmqhip.so python -u tools/gemm_sweep.py --tiles 0,1 > gpurun_out/ab_sweep_base.txt 2>&1 || { echo SWEEP_BASE_FAIL; exit 1; }
timeout -k 10 120 python -u tools/gemm_sweep.py --tiles 0,1 > gpurun_out/ab_sweep_new.txt 2>&1 || { echo SWEEP_NEW_FAIL; exit 1; }
timeout -k 10 300 env MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$PWD/tools/base_libmqhip.so python -u bench.py --no-cpu-baseline > gpurun_out/ab_bench_base.json 2> gpurun_out/ab_bench_base.err || { echo BENCH_BASE_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/ab_bench_new.json 2> gpurun_out/ab_bench_new.err || { echo BENCH_NEW_FAIL; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_gpu_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
echo AB_OK
