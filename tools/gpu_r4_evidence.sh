#!/bin/bash
# Round-4 evidence session (GPU box, repo root): same-box A/B of the round-3 library
# (variants/r3.so) vs the tree on the short bench, the MQ_KTRACE phase trace of the
# few-row kernels, the N=2 rehearsal (two ranks on one GPU, gloo), then the rocprofv3
# trace + PMC passes (profiles/run_profiles.sh).  First failure ends the script.
set -o pipefail
mkdir -p gpurun_out
SB="--steps 20 --warmup 3 --no-cpu-baseline --no-extras --config4-steps 0 --secondary-seq-len 0 --single-iters 30"
if [ -z "$SKIP_AB" ]; then
  for v in r3 new r3 new; do
    if [ $v = r3 ]; then L=$PWD/variants/r3.so; else L=$PWD/mediquery-rag_amd/mediquery_hip/libmqhip.so; fi
    timeout -k 10 300 env MQ_LIB_ALLOW_MISSING=1 MQ_LIB_PATH=$L python -u bench.py $SB >> gpurun_out/ab_r3_$v.jsonl 2>> gpurun_out/ab_r3.err || { echo AB_FAIL $v; tail -5 gpurun_out/ab_r3.err; exit 1; }
  done
  python - <<'PY'
import json
for v in ("r3", "new"):
    for l in open("gpurun_out/ab_r3_%s.jsonl" % v):
        d = json.loads(l)
        print(v, d["value"], d["ms_per_step"], d["encoder_ms"], d["search_ms"], d["kernels"]["flat_search_kernel"]["ms_per_step"], d["p50_single_query_ms"])
PY
fi
if [ -z "$SKIP_KT" ]; then
  MQ_LIB_PATH=$PWD/variants/ktrace.so timeout -k 5 150 python -u tools/ktrace.py > gpurun_out/ktrace_L32.txt 2>&1 || { echo KT_FAIL; tail -5 gpurun_out/ktrace_L32.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/ktrace_L32.txt | head -40
fi
if [ -z "$SKIP_N2" ]; then
  bash tools/rehearse_n2.sh || { echo N2_FAIL; tail -5 gpurun_out/bench_n2.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_n2.json'));print('N2', d['value'], d['n_gpus'], d['planted_top1_ok'])"
fi
if [ -z "$SKIP_PROF" ]; then
  bash profiles/run_profiles.sh r4 || { echo PROF_FAIL; exit 1; }
fi
echo EVIDENCE_OK
