set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_filter.py tests/test_gpu_store.py tests/test_gpu_index.py tests/test_gpu_i8.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1 && \
timeout -k 10 120 ./tools/engine_probe > gpurun_out/engine_probe.jsonl 2>&1
