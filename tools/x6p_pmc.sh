#!/bin/bash
# PMC passes over the K2p GEMM variants (run via gpurun from the repo root):
#   bash tools/x6p_pmc.sh <tag> <shape> <x6p tiles> [f32 tiles]
# Kernel trace first, then one counter group per pass (never mixed with trace domains).
# Summary: python3 tools/x6p_pmc_summary.py gpurun_out/x6p_pmc_<tag>
set -euo pipefail
TAG=${1:-a}; SHAPE=${2:-ffn_up}; TILES=${3:-0,4}; F32=${4:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/x6p_pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD="$ROOT/tools/gemm_x6p_bench.py --shapes $SHAPE --x6p-tiles=$TILES --f32-tiles=$F32 --iters 5 --reps 1"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $CMD > "$OUT/trace.txt" 2> "$OUT/trace.err"
echo trace done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run -- python3 $CMD > "$OUT/sq.txt" 2> "$OUT/sq.err"
echo sq done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq2" -o run -- python3 $CMD > "$OUT/sq2.txt" 2> "$OUT/sq2.err" || echo sq2 failed
echo sq2 done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE --output-format csv -d "$OUT/tcc" -o run -- python3 $CMD > "$OUT/tcc.txt" 2> "$OUT/tcc.err"
echo tcc done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $CMD > "$OUT/fetch.txt" 2> "$OUT/fetch.err"
echo fetch done
