#!/bin/bash
# Same-box A/B of K2p builds: tools/gemm_x6p_bench.py (tile -1, the headline shapes) on the
# tree's library and abvar/<v>.so (VARIANTS), alternating, REPS rounds.
set -o pipefail
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for v in main $VARIANTS; do
    if [ $v = main ]; then L=$PWD/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$PWD/abvar/$v.so; fi
    MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L timeout -k 10 200 python -u tools/gemm_x6p_bench.py --f32-tiles "" --x6p-tiles -1 \
      > gpurun_out/abx_${v}_$rep.jsonl 2>&1 || { echo FAIL $v; tail -5 gpurun_out/abx_${v}_$rep.jsonl; exit 1; }
    echo "== $v $rep"; grep '"us"' gpurun_out/abx_${v}_$rep.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], d['us'], d['frac_417'])"
  done
done
echo ABX_OK
