set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 env MQ_LIB_PATH=$PWD/tools/base_libmqhip.so python -u tools/gemm_sweep.py --shapes ffn_up --tiles 0,1 --epi 0 > gpurun_out/ab_sweep_base_epi0.txt 2>&1 || { echo SWEEP0_FAIL; exit 1; }
bash tools/ab_gemm.sh
