#!/bin/bash
# Short-bench A/B of the in-tree library against variants/<name>.so (VARIANTS="a b"),
# alternating, on one box; prints the encoder kernel classes per run.
set -o pipefail
mkdir -p gpurun_out
SB="--steps 20 --warmup 3 --no-cpu-baseline --no-extras --config4-steps 0 --secondary-seq-len 0 --single-iters 10 $BENCH_ARGS"
for rep in 1 2; do
  for v in main $VARIANTS; do
    if [ $v = main ]; then L=$PWD/mediquery-rag_amd/mediquery_hip/libmqhip.so; else L=$PWD/variants/$v.so; fi
    timeout -k 10 300 env MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L python -u bench.py $SB >> gpurun_out/abv_$v.jsonl 2>> gpurun_out/abv.err || { echo AB_FAIL $v; tail -5 gpurun_out/abv.err; exit 1; }
  done
done
python - <<'PY'
import json, os
for v in ["main"] + os.environ.get("VARIANTS", "").split():
    for l in open("gpurun_out/abv_%s.jsonl" % v):
        d = json.loads(l); k = d["kernels"]
        print(v, d["value"], d["ms_per_step"], {n: k[n]["ms_per_step"] for n in ("qkv_gemm", "out_proj_gemm", "layernorm", "ffn_up_gemm", "ffn_down_gemm", "attention")})
PY
echo ABV_OK
