# r6: survivor select with the thread-maxima cut - search tests, then kernel traces of the
# product library and of the committed select (tools/abvar/selold.so) on the same box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_thresh.py tests/test_gpu_i8.py tests/test_gpu_filter.py tests/test_gpu_index.py tests/test_gpu_single_clustered.py > gpurun_out/select_tests.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/select_prof -o run -- python3 -u tools/thresh_bench.py --iters 30 > gpurun_out/select_bench.log 2>&1 &&
MQ_LIB_PATH=$PWD/tools/abvar/selold.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/select_old -o run -- python3 -u tools/thresh_bench.py --iters 30 > gpurun_out/select_old.log 2>&1
