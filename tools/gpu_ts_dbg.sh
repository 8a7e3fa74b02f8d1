#!/bin/bash
# K9t bound decomposition: the tree against -DMQ_TS_DBG variants (measurement builds; their
# tau is +inf so the garbage scores append nothing), kernel trace of tools/thresh_bench.py.
set -o pipefail
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
for v in main $TS_VARIANTS; do
  if [ $v = main ]; then L=$R/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$R/variants/$v.so; fi
  MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tsd_$v -o run -- python3 $R/tools/thresh_bench.py --batches 256,1024 --iters 10 > $R/gpurun_out/tsd_$v.txt 2>&1 || { echo TSV_FAIL $v; tail -5 $R/gpurun_out/tsd_$v.txt; exit 1; }
done
cd $R && for v in main $TS_VARIANTS; do echo "== $v"; python3 tools/trace_summary.py gpurun_out/tsd_$v | grep -i "thresh"; done
echo TSD_OK
