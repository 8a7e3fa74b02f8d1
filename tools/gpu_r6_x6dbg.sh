# r6: price the parts of the K2p k-step (measurement build, wrong results): tile 0 vs no split
# (12), no A fragment reads (14), no W3 fragment reads (13), no fragment reads (10)
set -o pipefail
mkdir -p gpurun_out
MQ_LIB_PATH=$PWD/tools/abvar/x6dbg.so timeout -k 10 600 python -u tools/gemm_x6p_bench.py --f32-tiles "" --x6p-tiles=0,12,14,13,10 --iters 20 --reps 5 > gpurun_out/x6dbg.jsonl 2> gpurun_out/x6dbg.err
