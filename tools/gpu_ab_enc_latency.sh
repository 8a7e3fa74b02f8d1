#!/bin/bash
# Single-query encoder latency A/B: the tree vs variants/<v>.so (VARIANTS), alternating
# tools/latency.py runs (encoder p50 at several token counts, then end to end); TESTS first.
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/abe_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/abe_tests.log; exit 1; }
  tail -1 gpurun_out/abe_tests.log
fi
for rep in 1 2 3; do
  for v in main $VARIANTS; do
    if [ $v = main ]; then L=$PWD/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$PWD/variants/$v.so; fi
    MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L timeout -k 10 200 python -u tools/latency.py --encoder-seq-lens ${LENS:-16,32,64} --iters 300 > gpurun_out/abe_${v}_$rep.txt 2>&1 || { echo LAT_FAIL $v; tail -5 gpurun_out/abe_${v}_$rep.txt; exit 1; }
    echo "$v $rep $(tail -1 gpurun_out/abe_${v}_$rep.txt)"
  done
done
echo ABE_OK
