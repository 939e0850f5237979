#!/bin/bash
# Session-3: 2-rank rehearsals on one GPU (gloo: more ranks than GPUs) of the
# genome and shard modes on the final build.
set -e
O=gpurun_out/s3ranks
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 2 --scale 0.05 --steps 3 --warmup 1 --no-cpu --out $O/genome2.json > $O/genome2.log 2>&1
timeout -k 10 400 python bench.py --gpus 2 --mode shard --scale 0.05 --steps 3 --warmup 1 --no-cpu --out $O/shard2.json > $O/shard2.log 2>&1
