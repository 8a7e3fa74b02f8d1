#!/bin/bash
# PMC passes over selected GEMM tiles (run via gpurun from the repo root):
#   bash tools/gemm_pmc.sh <tag> <shapes> <tiles>
set -euo pipefail
TAG=${1:-g}; SHAPES=${2:-qkv,ffn_up}; TILES=${3:-1,6}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD="$ROOT/tools/gemm_sweep.py --shapes $SHAPES --tiles $TILES --iters 5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run -- python3 $CMD > "$OUT/sq.txt" 2> "$OUT/sq.err"
echo sq done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr GRBM_GUI_ACTIVE --output-format csv -d "$OUT/tcc" -o run -- python3 $CMD > "$OUT/tcc.txt" 2> "$OUT/tcc.err"
echo tcc done
