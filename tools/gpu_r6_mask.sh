# r6: masked K9t without per-block mask terms (no spill) - filter / search tests, then the
# filtered-search latency line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_filter.py tests/test_gpu_thresh.py tests/test_gpu_store.py tests/test_gpu_index.py > gpurun_out/mask_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/filter_latency.py > gpurun_out/mask_filter_latency.json 2> gpurun_out/mask_filter_latency.err
