#!/bin/bash
# Encoder A/B on one box: GPU encoder tests, then the short bench alternating an encoder
# option (ENC_OPT, e.g. ln_on_load=0) against the default build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_encoder.py} -x -q --timeout 200 --timeout-method thread > gpurun_out/enc_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/enc_tests.log; exit 1; }
tail -1 gpurun_out/enc_tests.log
SB="--steps 20 --warmup 3 --no-cpu-baseline --no-extras --config4-steps 0 --secondary-seq-len 0 --single-iters 20"
for v in new opt new opt; do
  if [ $v = opt ]; then O="--enc-opt $ENC_OPT"; else O=""; fi
  timeout -k 10 300 python -u bench.py $SB $O >> gpurun_out/ab_enc_$v.jsonl 2>> gpurun_out/ab_enc.err || { echo AB_FAIL $v; tail -5 gpurun_out/ab_enc.err; exit 1; }
done
python - <<'PY'
import json
for v in ("new", "opt"):
    for l in open("gpurun_out/ab_enc_%s.jsonl" % v):
        d = json.loads(l); k = d["kernels"]
        print(v, d["value"], d["ms_per_step"], d["encoder_ms"], {n: k[n]["ms_per_step"] for n in ("qkv_gemm", "out_proj_gemm", "layernorm", "ffn_up_gemm", "ffn_down_gemm")})
PY
echo AB_OK
