#!/bin/bash
# Named GPU test files first (NEW_TESTS), then the whole GPU suite and smoke().
set -o pipefail
mkdir -p gpurun_out
if [ -n "$NEW_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $NEW_TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { echo NEW_TESTS_FAIL; tail -30 gpurun_out/new_tests.log; exit 1; }
  tail -1 gpurun_out/new_tests.log
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
echo ALL_OK
