#!/bin/bash
# End-of-round evidence on one MI355X: default N=1 bench (the driver's command), then the
# round's rocprofv3 passes (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ) and a
# single-query latency sweep by token count.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo BENCH_FAIL; tail -5 gpurun_out/bench_final.err; exit 1; }
echo BENCH_OK
bash profiles/run_profiles.sh r3 || { echo PROF_FAIL; exit 1; }
timeout -k 10 200 python -u tools/latency.py --iters 100 --encoder-seq-lens 16,32,64,128,256,512 > gpurun_out/lat_final.json 2>&1 || { echo LAT_FAIL; exit 1; }
echo ALL_OK
