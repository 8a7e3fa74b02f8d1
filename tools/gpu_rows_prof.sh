# Kernel-trace the single-query latency tool with the few-row forward on and off.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/enc_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/enc_tests.log; exit 1; }
tail -1 gpurun_out/enc_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_rows -o run -- python3 $ROOT/tools/latency.py --iters 100 > $ROOT/gpurun_out/prof_rows.log 2>&1 || { echo P1_FAIL; exit 1; }
env ${BENV:-MQ_ROWS_PATH=0} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_old -o run -- python3 $ROOT/tools/latency.py --iters 100 > $ROOT/gpurun_out/prof_old.log 2>&1 || { echo P2_FAIL; exit 1; }
echo DONE
