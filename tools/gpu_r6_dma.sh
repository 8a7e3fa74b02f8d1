# r6: K9t A/B - which waves issue the ring's DMAs: all 8 (MQ_TS_DMAW=8) vs waves 0-3 / 0-1 / 0
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dma_base -o run -- python3 -u tools/thresh_bench.py --iters 30 > gpurun_out/dma_base.log 2>&1 &&
for w in 4 2 1; do
  MQ_LIB_PATH=$PWD/tools/abvar/tsdma$w.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dma_$w -o run -- python3 -u tools/thresh_bench.py --iters 30 > gpurun_out/dma_$w.log 2>&1 || exit 1
done
