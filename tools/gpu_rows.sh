set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/enc_tests.log; exit 1; }
tail -2 gpurun_out/enc_tests.log
timeout -k 10 200 python -u tools/latency.py --iters 200 > gpurun_out/lat_rows.json 2>&1 || { echo LAT_FAIL; exit 1; }
MQ_ROWS_PATH=0 timeout -k 10 200 python -u tools/latency.py --iters 200 > gpurun_out/lat_old.json 2>&1 || { echo LAT0_FAIL; exit 1; }
cat gpurun_out/lat_rows.json; echo; cat gpurun_out/lat_old.json
