#!/bin/bash
# Collect the rocprofv3 evidence for one round on the GPU box (run via gpurun from the
# repo root).  Kernel trace + stats first, then one PMC pass per TCC counter (FETCH_SIZE
# and WRITE_SIZE do not fit one pass on gfx950), never mixed with trace domains.
set -euo pipefail
R=${1:-r1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --single-iters 10"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch_bench.json" 2> "$OUT/fetch.err"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write_bench.json" 2> "$OUT/write.err"
echo "profiles done"
