# r6: few-row plane merge - encoder parity, single-query latency A/B (rows_planes 0 / 1, alternating)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t6_enc.log 2>&1 && \
timeout -k 10 400 python -u tools/latency.py --iters 200 --e2e-opt rows_planes=0,1,0,1,0 > gpurun_out/t6_latency_ab.txt 2>&1 && \
timeout -k 10 300 python -u tools/latency.py --iters 200 > gpurun_out/t6_latency.txt 2>&1
