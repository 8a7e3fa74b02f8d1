#!/bin/bash
# r3 evidence: the round's rocprofv3 passes over the bench, then a kernel trace of
# single-query forwards at L = 256 (advisor-length queries).
set -o pipefail
mkdir -p gpurun_out
bash profiles/run_profiles.sh r3 || { echo PROF_FAIL; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/l256_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/latency.py --iters 30 --encoder-seq-lens 256 > $GRAFT_REPO_ROOT/gpurun_out/l256_prof.log 2>&1 || { echo L256_FAIL; exit 1; }
echo ALL_OK
