#!/bin/bash
# Long single queries on the tiled path: encoder option tests, then p50 by token count for a
# sweep of MQ_ENC_OPT_SPLITK_TILES (which GEMMs of an M <= 256 forward split over K).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-sk}
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -k "options" -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u tools/latency.py --iters 100 --encoder-seq-lens 96,128,192,256 --opt splitk_tiles=${VALS:-0,192,128,96,64,32} > gpurun_out/${TAG}_lens.json 2>&1 || { echo LENS_FAIL; tail -5 gpurun_out/${TAG}_lens.json; exit 1; }
tail -1 gpurun_out/${TAG}_lens.json
echo ALL_OK
