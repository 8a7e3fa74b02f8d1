# r6: few-row frag16 layout check - encoder parity tests, smoke, single-query latency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t3_enc.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t3_smoke.log 2>&1 && \
timeout -k 10 300 python -u tools/latency.py --iters 200 > gpurun_out/t3_latency.txt 2>&1
