# r6: region tile walks - GEMM / encoder parity, then the bench line (kernel classes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_gemm_x6p.py tests/test_gpu_encoder.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t5_tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --config4-steps 0 > gpurun_out/t5_bench.json 2> gpurun_out/t5_bench.err
