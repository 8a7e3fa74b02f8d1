# Round-end style check on one MI355X: GPU tests, smoke, N=1 bench, single-query latency.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 200 python -u tools/latency.py --iters 200 > gpurun_out/lat.json 2>&1 || { echo LAT_FAIL; exit 1; }
timeout -k 10 420 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
