set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/gemm_sweep.py --tiles 0,1 > gpurun_out/sw_main.txt 2>&1 || exit 1
timeout -k 10 120 env MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$PWD/variants/nostore.so python -u tools/gemm_sweep.py --tiles 0,1 > gpurun_out/sw_nostore.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/gemm_sweep.py --tiles 0,1 > gpurun_out/sw_main2.txt 2>&1 || exit 1
echo SW_OK
