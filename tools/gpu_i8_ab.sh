#!/bin/bash
# int8 single-query screen (K9q): parity tests, then single-query latency of the in-tree
# library vs variants/*.so (same box, alternating).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_thresh.py -x -q --timeout 200 --timeout-method thread > gpurun_out/i8_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/i8_tests.log; exit 1; }
tail -1 gpurun_out/i8_tests.log
for r in 1 2; do
  timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/i8_lat_new_$r.json 2>&1 || { echo LAT_FAIL; tail -5 gpurun_out/i8_lat_new_$r.json; exit 1; }
  tail -1 gpurun_out/i8_lat_new_$r.json
  MQ_LIB_PATH=$PWD/variants/base.so timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/i8_lat_base_$r.json 2>&1 || { echo LAT_FAIL; exit 1; }
  tail -1 gpurun_out/i8_lat_base_$r.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/i8_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/latency.py --iters 100 > $GRAFT_REPO_ROOT/gpurun_out/i8_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
