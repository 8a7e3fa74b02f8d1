# Few-row FFN-down K splits (MQ_ROWS_SPLITS = 2 / 3 / 4): encoder tests at 2, then the
# single-query encoder p50 and per-kernel rocprof averages for each setting.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
MQ_ROWS_SPLITS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_encoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sp_t.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/sp_t.log; exit 1; }
tail -1 gpurun_out/sp_t.log
for sp in 2 3 4; do
  MQ_ROWS_SPLITS=$sp timeout -k 10 120 python -u tools/latency.py --iters 300 --encoder-seq-lens 32 > gpurun_out/sp_lat$sp.txt 2>&1 || { echo LAT_FAIL $sp; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
for sp in 2 3 4; do
  MQ_ROWS_SPLITS=$sp timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/sp_prof$sp -o run -- python3 $ROOT/tools/latency.py --iters 100 --encoder-seq-lens 32 > $ROOT/gpurun_out/sp_prof$sp.log 2>&1 || { echo PROF_FAIL $sp; exit 1; }
done
echo SP_OK
