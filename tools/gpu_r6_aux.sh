# r6 evidence: filtered-search / delete latency at 1M rows, LangChain-level latency, and the
# N = 2 rehearsal (two gloo ranks on the one GPU) with the distributed fields of the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/filter_latency.py > gpurun_out/filter_latency_1m.json 2> gpurun_out/filter_latency.err && \
timeout -k 10 300 python -u tools/langchain_latency.py > gpurun_out/langchain_latency.txt 2>&1 && \
bash tools/rehearse_n2.sh
