#!/bin/bash
# Single-query latency check on one MI355X: few-row parity tests, p50 by token count,
# and a kernel trace of the L=32 single-query encoder (per-launch durations).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-lat}
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py ${EXTRA_TESTS} -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u tools/latency.py --iters 200 > gpurun_out/${TAG}_l32.json 2>&1 || { echo LAT_FAIL; tail -5 gpurun_out/${TAG}_l32.json; exit 1; }
tail -1 gpurun_out/${TAG}_l32.json
timeout -k 10 200 python -u tools/latency.py --iters 100 --encoder-seq-lens 16,32,48,64,96,128,256,512 > gpurun_out/${TAG}_lens.json 2>&1 || { echo LENS_FAIL; exit 1; }
tail -1 gpurun_out/${TAG}_lens.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/latency.py --iters 50 --encoder-seq-lens ${PROF_LENS:-32} > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
