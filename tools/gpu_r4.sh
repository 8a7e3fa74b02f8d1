#!/bin/bash
# Round-4 GPU session: named new test files, the whole GPU suite, smoke(), the bench,
# and a single-query latency A/B of tools/base_libmqhip.so (previous build) vs the tree.
# Run from the repo root on the GPU box.  Every GPU step has its own time limit; the
# first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step new_tests
timeout -k 10 600 python -u -m pytest ${NEW_TESTS:-tests/test_gpu_screen_cost.py} -x -v -s --timeout 200 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { echo NEW_TESTS_FAIL; tail -40 gpurun_out/new_tests.log; exit 1; }
tail -1 gpurun_out/new_tests.log
if [ -z "$SKIP_SUITE" ]; then
  step suite
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [ -z "$SKIP_BENCH" ]; then
  step bench
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['p50_single_query_ms'],d['roofline']['frac'])"
fi
if [ -n "$AB_LATENCY" ] && [ -f tools/base_libmqhip.so ]; then
  step ab_latency
  for v in base new base new; do
    if [ $v = base ]; then L=$PWD/tools/base_libmqhip.so; else L=$PWD/mediquery-rag_amd/mediquery_hip/libmqhip.so; fi
    timeout -k 10 200 env MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L python -u tools/latency.py --iters 300 >> gpurun_out/ab_latency_$v.txt 2>&1 || { echo LAT_FAIL; exit 1; }
  done
  tail -5 gpurun_out/ab_latency_base.txt gpurun_out/ab_latency_new.txt
fi
echo ALL_OK
