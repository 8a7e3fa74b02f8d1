#!/bin/bash
# Rehearse the N=2 bench path on a one-GPU box (both ranks on cuda:0, gloo for the
# collectives) - the driver runs the real N>1 benches on an 8-GPU node.
set -o pipefail
mkdir -p gpurun_out
MQ_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-cpu-baseline --single-iters 5 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
