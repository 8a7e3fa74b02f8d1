# r6: FETCH_SIZE per K2p launch by tile-walk region split (rx), FFN-up and QKV shapes
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/rx_pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $ROOT/gpurun_out/rx_pmc/fetch -o run -- python3 $ROOT/tools/gemm_x6p_bench.py --shapes ffn_up,qkv --f32-tiles= --x6p-tiles=100,200,300,500,900 --iters 5 --reps 1 > $ROOT/gpurun_out/rx_pmc/bench.jsonl 2> $ROOT/gpurun_out/rx_pmc/err.txt
