#!/bin/bash
# Final-build evidence of a session: GPU tests, smoke, the default bench line,
# a rocprofv3 kernel trace (stats + step timeline) and the PMC passes
# (tools/gpu_pmc.sh) of the same build; the profiled runs skip the visits
# line (its scans run beside a concurrent count and would mix into the averages).  Usage: tools/s3_final.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -20 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
timeout -k 10 400 python bench.py --out $O/bench.json > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --no-visits > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
cd $R
bash tools/gpu_pmc.sh $TAG --no-visits
