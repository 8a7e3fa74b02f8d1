#!/bin/bash
# BASELINE §8f row 3 at full size: 1M documents through HipBertEmbeddings.embed_array + FlatIndex.add
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ingest_bench.py --docs 1000000 > gpurun_out/ingest_1m.json 2> gpurun_out/ingest_1m.err || { echo INGEST_FAIL; tail -5 gpurun_out/ingest_1m.err; exit 1; }
cat gpurun_out/ingest_1m.json
echo ALL_OK
