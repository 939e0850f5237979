#!/bin/bash
# Round-2 GPU session: the -m gpu suite, then bench lines (metric config with
# its parity sample, weighted rank, host entry point with visits).
# Usage: tools/gpu_r2.sh TAG [pytest -k expr]
set -o pipefail
TAG=$1; KEXPR=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ -n "$KEXPR" ]; then KARG=(-k "$KEXPR"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -3 $OUT/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --out $OUT/bench_$TAG.json > $OUT/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench_$TAG.log; exit 1; }
cat $OUT/bench_$TAG.json
timeout -k 10 300 python bench.py --score rank --steps 3 --out $OUT/rank_$TAG.json > $OUT/rank_$TAG.log 2>&1 || { echo "rank bench failed"; tail -30 $OUT/rank_$TAG.log; exit 1; }
cat $OUT/rank_$TAG.json
timeout -k 10 300 python bench.py --host-path --no-cpu --steps 3 --out $OUT/host_$TAG.json > $OUT/host_$TAG.log 2>&1 || { echo "host bench failed"; tail -30 $OUT/host_$TAG.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/host_$TAG.json')); print('host_path', d['host_path'])"
