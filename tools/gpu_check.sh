#!/bin/bash
# One GPU session: the -m gpu suite, the default bench line, and a 2-rank
# gloo rehearsal of the multi-rank launcher on the one GPU of the box.
# Usage: tools/gpu_check.sh TAG [extra pytest args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -3 $OUT/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --out $OUT/bench_$TAG.json > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_$TAG.log; exit 1; }
cat $OUT/bench_$TAG.json
timeout -k 10 300 python bench.py --gpus 2 --scale 0.05 --steps 3 --out $OUT/bench2_$TAG.json > $OUT/bench2_$TAG.log 2>&1 || { echo "bench --gpus 2 failed"; tail -30 $OUT/bench2_$TAG.log; exit 1; }
cat $OUT/bench2_$TAG.json
