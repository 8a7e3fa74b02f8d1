#!/bin/bash
# K9t A/B: the tree vs variants/<v>.so (VARIANTS), alternating, kernel trace of
# tools/thresh_bench.py (B = 256 and 1024 over 1M rows); then the screen / thresh tests.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_thresh.py tests/test_gpu_screen_cost.py tests/test_gpu_index.py > gpurun_out/abt_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/abt_tests.log; exit 1; }
tail -1 gpurun_out/abt_tests.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in main $VARIANTS; do
    if [ $v = main ]; then L=$R/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$R/variants/$v.so; fi
    MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/abt_${v}_$rep -o run -- python3 $R/tools/thresh_bench.py --batches 256,1024 --iters 10 > $R/gpurun_out/abt_${v}_$rep.txt 2>&1 || { echo ABT_FAIL $v; tail -5 $R/gpurun_out/abt_${v}_$rep.txt; exit 1; }
  done
done
cd $R && for rep in 1 2; do for v in main $VARIANTS; do echo "== $v $rep"; python3 tools/trace_summary.py gpurun_out/abt_${v}_$rep | grep -i "thresh_kernel"; done; done
echo ABT_OK
