#!/bin/bash
# Encoder parity tests + single-query latency breakdown (tools/latency.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 200 python -u tools/latency.py > gpurun_out/latency_new.txt 2>&1 || { echo LAT_FAIL; exit 1; }
echo OK
