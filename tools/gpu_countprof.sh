#!/bin/bash
# Count parity tests, the in-process count timing and a kernel trace of it.
# Usage: tools/gpu_countprof.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "count or Count" > $O/pytest_count.txt 2>&1 || { tail -30 $O/pytest_count.txt; exit 1; }
tail -1 $O/pytest_count.txt
timeout -k 10 300 python tools/ab_count.py --k 13 --rounds 3 base: > $O/count_ab.txt 2>&1 || { tail -20 $O/count_ab.txt; exit 1; }
tail -2 $O/count_ab.txt
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o cnt --output-format csv -- python3 $R/tools/ab_count.py --k 13 --rounds 1 --steps 3 base: > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'ks::' in r['Name']:
        print(f"{int(r['Calls']):4d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:70]}")
PY
