#!/bin/bash
# Single-query latency A/B: the tree vs variants/<v>.so (VARIANTS), alternating runs of
# tools/latency.py over a 1M-row corpus; TESTS (optional) run first on the tree.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/abl_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/abl_tests.log; exit 1; }
  tail -1 gpurun_out/abl_tests.log
fi
for rep in 1 2 3; do
  for v in main $VARIANTS; do
    if [ $v = main ]; then L=$PWD/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$PWD/variants/$v.so; fi
    MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L timeout -k 10 200 python -u tools/latency.py --iters 300 $LAT_ARGS > gpurun_out/abl_${v}_$rep.txt 2>&1 || { echo LAT_FAIL $v; tail -5 gpurun_out/abl_${v}_$rep.txt; exit 1; }
    python3 -c "
import ast,sys; d=ast.literal_eval(open('gpurun_out/abl_${v}_$rep.txt').read().strip().splitlines()[-1])
print('$v', $rep, 'search', d['search_ms'], 'e2e', d['end_to_end_ms'], 'enc', d['encoder_ms'], d['search_stage_ms'])"
  done
done
echo ABL_OK
