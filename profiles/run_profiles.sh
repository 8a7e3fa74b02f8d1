#!/bin/bash
# Collect the rocprofv3 evidence for one round on the GPU box (run via gpurun from the
# repo root).  Kernel trace + stats first, then one PMC pass per counter group, never
# mixed with trace domains (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
# Summaries: python3 tools/summarize_profiles.py gpurun_out/prof_<round> profiles/<round>
set -euo pipefail
R=${1:-r2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --single-iters 10 --secondary-seq-len 0 --config4-steps 0 --no-extras"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
echo "trace done"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch_bench.json" 2> "$OUT/fetch.err"
echo "fetch done"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write_bench.json" 2> "$OUT/write.err"
echo "write done"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o run -- python3 $BENCH > "$OUT/sq_bench.json" 2> "$OUT/sq.err"
echo "profiles done"
