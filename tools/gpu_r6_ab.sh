# r6: same-box A/B of library variants on the bench's short line (kernel breakdown per variant)
# usage: bash tools/gpu_r6_ab.sh name1 name2 ...   (name "base" = the product library)
set -o pipefail
mkdir -p gpurun_out/ab
B="bench.py --steps 20 --warmup 3 --no-cpu-baseline --single-iters 10 --secondary-seq-len 0 --config4-steps 0 --no-extras"
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/tools/abvar/$v.so; fi
  MQ_LIB_PATH=$lib timeout -k 10 300 python -u $B > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
done
