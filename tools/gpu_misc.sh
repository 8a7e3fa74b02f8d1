#!/bin/bash
# r3: encoder tests (attention change), N=1 bench, ingest at scale, filtered-search latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py tests/test_gpu_gemm.py tests/test_gpu_store.py -x -q --timeout 200 --timeout-method thread > gpurun_out/misc_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/misc_tests.log; exit 1; }
tail -1 gpurun_out/misc_tests.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -5 gpurun_out/bench.err; exit 1; }
echo BENCH_OK
timeout -k 10 300 python -u tools/filter_latency.py > gpurun_out/filter.json 2> gpurun_out/filter.err || { echo FILTER_FAIL; tail -5 gpurun_out/filter.err; exit 1; }
cat gpurun_out/filter.json
timeout -k 10 560 python -u tools/ingest_bench.py --docs ${INGEST_DOCS:-1000000} > gpurun_out/ingest.json 2> gpurun_out/ingest.err || { echo INGEST_FAIL; tail -5 gpurun_out/ingest.err; exit 1; }
cat gpurun_out/ingest.json
