# r6: the default bench line alone (after a profile refresh)
set -o pipefail
mkdir -p gpurun_out/r6bench
timeout -k 10 500 python -u bench.py > gpurun_out/r6bench/bench_n1.json 2> gpurun_out/r6bench/bench_n1.err
