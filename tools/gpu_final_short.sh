#!/bin/bash
# Short end-of-round check at HEAD: full GPU suite, smoke(), default bench, single-query p50.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo BENCH_FAIL; tail -5 gpurun_out/bench_final.err; exit 1; }
echo BENCH_OK
echo FINAL_OK
