# r6: ktrace of the few-row kernels (measurement variant), encoder parity, short bench
set -o pipefail
mkdir -p gpurun_out
MQ_LIB_PATH=tools/variants/ktrace.so timeout -k 10 200 python -u tools/ktrace.py > gpurun_out/t4_ktrace.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t4_enc.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline --config4-steps 0 --secondary-seq-len 0 > gpurun_out/t4_bench.json 2> gpurun_out/t4_bench.err
