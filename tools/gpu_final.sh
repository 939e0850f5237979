#!/bin/bash
# Round-end evidence of the current build: GPU tests, the default bench line,
# a rocprofv3 kernel trace + stats of the metric step, and the PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs, kernel records only) that
# profiles/pmc_summary.json is assembled from.  Usage: tools/jobs/final.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 600 python bench.py --out $O/bench.json > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
python -c "import json;b=json.load(open('$O/bench.json'));print('bench', b['value'], b['ms_per_step'], b['roofline']['frac'], b['parity_sample'], b['parity_bp'], (b.get('host_path') or {}).get('Gbases_per_s'), (b.get('configs') or {}).get('rank', {}).get('value'))"
B="--no-cpu --no-rank --no-host-path --no-visits"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 $B --out $O/prof_bench.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/step_timeline.txt || true
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B --out $O/pmc_bench.json > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $B > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
cd $R
python3 tools/pmc_assemble.py $O/pmc_bench.json $O/pmc_summary.json $(find $O/pmc_fetch $O/pmc_write -name '*counter_collection.csv') > $O/pmc_assemble.txt 2>&1 || { tail -20 $O/pmc_assemble.txt; exit 1; }
head -30 $O/pmc_assemble.txt
find $O/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} sh -c 'head -15 {}'
