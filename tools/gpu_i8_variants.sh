#!/bin/bash
# int8 screen build variants (variants/*.so): parity tests per variant, then single-query
# latency, alternating in-tree / variants twice on the same box.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_thresh.py tests/test_gpu_index.py tests/test_gpu_store.py -x -q --timeout 200 --timeout-method thread > gpurun_out/iv_tests_main.log 2>&1 || { echo TESTS_FAIL main; tail -30 gpurun_out/iv_tests_main.log; exit 1; }
echo main $(tail -1 gpurun_out/iv_tests_main.log)
for v in variants/*.so; do
  n=$(basename $v .so)
  MQ_LIB_PATH=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_thresh.py -x -q --timeout 200 --timeout-method thread > gpurun_out/iv_tests_$n.log 2>&1 || { echo TESTS_FAIL $n; tail -30 gpurun_out/iv_tests_$n.log; exit 1; }
  echo $n $(tail -1 gpurun_out/iv_tests_$n.log)
done
for r in 1 2; do
  timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/iv_lat_main_$r.json 2>&1 || { echo LAT_FAIL; exit 1; }
  echo main $(tail -1 gpurun_out/iv_lat_main_$r.json | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d['search_ms'], d['end_to_end_ms'], d['search_stage_ms'])")
  for v in variants/*.so; do
    n=$(basename $v .so)
    MQ_LIB_PATH=$PWD/$v timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/iv_lat_${n}_$r.json 2>&1 || { echo LAT_FAIL $n; exit 1; }
    echo $n $(tail -1 gpurun_out/iv_lat_${n}_$r.json | python3 -c "import sys,ast; d=ast.literal_eval(sys.stdin.read()); print(d['search_ms'], d['end_to_end_ms'], d['search_stage_ms'])")
  done
done
echo ALL_OK
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/iv_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/latency.py --iters 100 > $GRAFT_REPO_ROOT/gpurun_out/iv_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo PROF_OK
