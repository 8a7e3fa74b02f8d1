# r6 checkpoint: the whole GPU suite, then the default bench line and its rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out/r6full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6full/gpu_tests.log 2>&1 && \
timeout -k 10 500 python -u bench.py > gpurun_out/r6full/bench_n1.json 2> gpurun_out/r6full/bench_n1.err
