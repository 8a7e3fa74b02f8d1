# Kernel-trace the single-query encoder for the in-tree library and variants/*.so builds
# (measurement builds, e.g. -DMQ_MEASUREMENT_BUILD -DMQ_ROWS_DBG=1): per-kernel durations under gpurun_out/pv_<name>.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/pv_main -o run -- python3 $ROOT/tools/latency.py --iters 100 --encoder-seq-lens 32 > $ROOT/gpurun_out/pv_main.log 2>&1 || { echo MAIN_FAIL; exit 1; }
for v in $ROOT/variants/*.so; do
  n=$(basename $v .so)
  MQ_LIB_PATH=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/pv_$n -o run -- python3 $ROOT/tools/latency.py --iters 100 --encoder-seq-lens 32 > $ROOT/gpurun_out/pv_$n.log 2>&1 || { echo FAIL $n; exit 1; }
done
echo PV_OK
