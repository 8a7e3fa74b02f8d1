#!/bin/bash
# The rerank-rounds branch built as variants/rr.so: search parity tests through it, then
# single-query latency vs the in-tree library (same box, alternating).
set -o pipefail
mkdir -p gpurun_out
MQ_LIB_PATH=$PWD/variants/rr.so timeout -k 10 400 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_thresh.py tests/test_gpu_index.py tests/test_gpu_store.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rr_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/rr_tests.log; exit 1; }
tail -1 gpurun_out/rr_tests.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/rr_lat_main_$r.json 2>&1 || { echo LAT_FAIL; exit 1; }
  MQ_LIB_PATH=$PWD/variants/rr.so timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/rr_lat_rr_$r.json 2>&1 || { echo LAT_FAIL; exit 1; }
  echo main $(tail -1 gpurun_out/rr_lat_main_$r.json | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d['search_ms'], d['end_to_end_ms'])")
  echo rr $(tail -1 gpurun_out/rr_lat_rr_$r.json | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d['search_ms'], d['end_to_end_ms'])")
done
echo RR_OK
