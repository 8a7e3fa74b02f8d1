#!/bin/bash
# Kernel-trace A/B of measurement variants: rocprofv3 --kernel-trace --stats of
# tools/latency.py (search only matters) for the tree's library and abvar/<v>.so (VARIANTS).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in main $VARIANTS; do
  if [ $v = main ]; then L=$PWD/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$PWD/abvar/$v.so; fi
  MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/kt_$v -o kt -- python3 -u tools/latency.py --iters 100 $LAT_ARGS > gpurun_out/kt_$v.log 2>&1 || { echo FAIL $v; exit 1; }
  echo "== $v"; grep -h "search_ms" gpurun_out/kt_$v.log | cut -c1-200
done
echo KT_OK
