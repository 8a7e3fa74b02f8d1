# r6: K9t A/B - s_setprio for the MFMA-only waves (prio1) or the DMA waves (prio2) of the
# append pass (an MQ_TS_PRIO build macro, measured without gain and removed:
# profiles/r6/k9t_setprio_ab.txt); kernel stats only
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base prio1 prio2 base2; do
  case $v in base|base2) lib="";; *) lib=$PWD/tools/abvar/$v.so;; esac
  MQ_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prio_$v -o run -- python3 -u tools/thresh_bench.py --iters 30 --batches 256 > gpurun_out/prio_$v.log 2>&1 || exit 1
  rm -f gpurun_out/prio_$v/run_kernel_trace.csv
done
