#!/bin/bash
# Memory-path PMC passes over K2p variants (run via gpurun from the repo root):
#   LIB=<.so or empty> bash tools/x6p_pmc2.sh <tag> <shape> <x6p tiles>
# One counter group per pass, each under its own kill timeout.
# Summary: python3 tools/x6p_pmc_summary.py gpurun_out/x6p_pmc_<tag>
set -uo pipefail
TAG=${1:-b}; SHAPE=${2:-ffn_up}; TILES=${3:-0,12}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/x6p_pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
if [ -n "${LIB:-}" ]; then export MQ_LIB_PATH=$LIB MQ_LIB_ALLOW_MISSING=1; fi
CMD="$ROOT/tools/gemm_x6p_bench.py --shapes $SHAPE --x6p-tiles=$TILES --f32-tiles= --iters 5 --reps 1"
run() {  # run <name> <counters...>
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$n" -o run -- python3 $CMD > "$OUT/$n.txt" 2> "$OUT/$n.err"
  local rc=$?
  echo "$n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $CMD > "$OUT/trace.txt" 2> "$OUT/trace.err" || exit 1
echo trace done
run p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VMEM GRBM_GUI_ACTIVE
run p2 SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run p3 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE
run p4 TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum
run p5 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_LEVEL_sum GRBM_GUI_ACTIVE
echo all done
