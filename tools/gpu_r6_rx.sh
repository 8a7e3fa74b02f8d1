# r6: K2p tile-walk region split (rx) sweep at the headline shapes, bit-identity vs the x6 tile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/gemm_x6p_bench.py --f32-tiles 5 --x6p-tiles=-1,100,200,300,500,900,107,207,307,507,907 --iters 20 --reps 5 > gpurun_out/rx_sweep.jsonl 2> gpurun_out/rx_sweep.err
