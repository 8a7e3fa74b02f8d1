#!/bin/bash
# End-of-round evidence at HEAD on one MI355X: the full GPU suite, smoke(), the default
# N=1 bench (the driver's command), the rocprofv3 passes and the latency-by-length sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final_gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo BENCH_FAIL; tail -5 gpurun_out/bench_final.err; exit 1; }
echo BENCH_OK
bash profiles/run_profiles.sh r3 || { echo PROF_FAIL; exit 1; }
timeout -k 10 200 python -u tools/latency.py --iters 100 --encoder-seq-lens 16,32,64,128,256,512 > gpurun_out/lat_final.json 2>&1 || { echo LAT_FAIL; exit 1; }
timeout -k 10 200 python -u tools/latency.py --iters 300 > gpurun_out/lat_final_l32.json 2>&1 || { echo LAT_FAIL; exit 1; }
echo FINAL_OK
