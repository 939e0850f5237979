#!/bin/bash
# Line tables: GPU tests, then the metric bench with line tables vs the J = 5 expanded table.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
for v in lines ext lines; do
  if [ $v = ext ]; then export KS_NO_LINES=1; else unset KS_NO_LINES; fi
  timeout -k 10 400 python bench.py --no-cpu --no-host-path --no-visits --no-rank --steps 10 --out $O/bench_$v.json > $O/bench_$v.log 2>&1 || { tail -30 $O/bench_$v.log; exit 1; }
  python -c "import json;b=json.load(open('$O/bench_$v.json'));print('$v',b['value'],b['ms_per_step'],b['phase_ms'],b['setup_ms'].get('table_ext_build'),b['config']['positions_per_read'])"
done
