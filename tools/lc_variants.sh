# LangChain-level single-query latency of the in-tree library and of variants/*.so builds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/langchain_latency.py --iters 200 > gpurun_out/lc_main.txt 2>&1 || { echo MAIN_FAIL; exit 1; }
for v in variants/*.so; do
  n=$(basename $v .so)
  MQ_LIB_PATH=$PWD/$v timeout -k 10 300 python -u tools/langchain_latency.py --iters 200 > gpurun_out/lc_$n.txt 2>&1 || { echo FAIL $n; exit 1; }
done
echo LC_OK
