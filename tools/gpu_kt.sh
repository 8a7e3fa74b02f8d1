#!/bin/bash
# few-row encoder: parity tests, L=32 latency, phase trace of the traced variant
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-kt}
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u tools/latency.py --iters 100 --encoder-seq-lens 32,64 > gpurun_out/${TAG}_lens.json 2>&1 || { echo LENS_FAIL; exit 1; }
tail -1 gpurun_out/${TAG}_lens.json
MQ_LIB_PATH=variants/ktrace.so timeout -k 5 150 python -u tools/ktrace.py > gpurun_out/${TAG}_ktrace.txt 2>&1 || { echo KT_FAIL; exit 1; }
cat gpurun_out/${TAG}_ktrace.txt | grep -v amdgpu.ids
