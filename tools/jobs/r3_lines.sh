#!/bin/bash
# r3: random whole-line read rates (tools/line_bench.hip) + a baseline bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3_lines
mkdir -p $O
cd $R
timeout -k 10 300 ./tools/line_bench 128 > $O/line_bench_128.txt 2>&1 || { cat $O/line_bench_128.txt; exit 1; }
cat $O/line_bench_128.txt
timeout -k 10 400 python bench.py --out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
cat $O/bench.json
