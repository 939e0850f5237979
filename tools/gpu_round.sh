#!/bin/bash
# One GPU session: parity tests, bench line, rocprofv3 kernel trace.
# Usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -3 $OUT/pytest_gpu_$TAG.log
timeout -k 10 600 python bench.py --out $OUT/bench_$TAG.json "$@" > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_$TAG.log; exit 1; }
cat $OUT/bench_$TAG.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu "$@" > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
find $OUT/prof_$TAG -name '*kernel_stats.csv' | head -1 | xargs -I{} sh -c 'head -12 {}'
