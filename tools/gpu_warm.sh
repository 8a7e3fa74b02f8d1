#!/bin/bash
# Spare-workgroup weight warm-up: encoder tests, single-query latency over warm_wgs, and the
# kernel trace of the few-row launches with and without spares; then the K9t TS_DBG variants.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > gpurun_out/warm_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/warm_tests.log; exit 1; }
tail -1 gpurun_out/warm_tests.log
for rep in 1 2; do
  timeout -k 10 200 python -u tools/latency.py --encoder-seq-lens 16,32,64 --opt warm_wgs=0,16,32,64,128 --iters 200 > gpurun_out/warm_lat_$rep.txt 2>&1 || { echo LAT_FAIL; tail -5 gpurun_out/warm_lat_$rep.txt; exit 1; }
  tail -1 gpurun_out/warm_lat_$rep.txt
done
timeout -k 10 200 python -u tools/latency.py --iters 200 > gpurun_out/warm_e2e.txt 2>&1 || { echo E2E_FAIL; exit 1; }
tail -1 gpurun_out/warm_e2e.txt
cd /tmp && export TMPDIR=/tmp
for w in 0 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/warm_trace_$w -o run -- python3 $R/tools/latency.py --encoder-seq-lens 32 --opt warm_wgs=$w --iters 50 > $R/gpurun_out/warm_tr_$w.txt 2>&1 || { echo TRACE_FAIL; exit 1; }
done
cd $R && python3 tools/trace_summary.py gpurun_out/warm_trace_0 gpurun_out/warm_trace_64 > gpurun_out/warm_trace_summary.txt && cat gpurun_out/warm_trace_summary.txt
if [ -n "$TS_VARIANTS" ]; then
  cd /tmp
  for v in main $TS_VARIANTS; do
    if [ $v = main ]; then L=$R/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$R/variants/$v.so; fi
    MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tsv_$v -o run -- python3 $R/tools/thresh_bench.py --batches 256 --iters 10 > $R/gpurun_out/tsv_$v.txt 2>&1 || { echo TSV_FAIL $v; tail -5 $R/gpurun_out/tsv_$v.txt; exit 1; }
  done
  cd $R && for v in main $TS_VARIANTS; do echo "== $v"; python3 tools/trace_summary.py gpurun_out/tsv_$v | grep -i "thresh"; done
fi
echo WARM_OK
