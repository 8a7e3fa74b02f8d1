# r6: K9t A/B - chain step of the DMA waves' first DMA (an MQ_TS_DMA_OFF build macro, measured
# without effect and removed: profiles/r6/k9t_dma_offset_ab.txt)
# kernel stats only (the full traces of five runs exceed what gpurun copies back)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base doff1 doff2 doff3 base2; do
  case $v in base|base2) lib="";; *) lib=$PWD/tools/abvar/$v.so;; esac
  MQ_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/doff_$v -o run -- python3 -u tools/thresh_bench.py --iters 30 --batches 256 > gpurun_out/doff_$v.log 2>&1 || exit 1
  rm -f gpurun_out/doff_$v/run_kernel_trace.csv
done
