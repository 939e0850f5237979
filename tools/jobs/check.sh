#!/bin/bash
# GPU tests + the default bench line of the current build.  Usage: tools/jobs/check.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 600 python bench.py --out $O/bench.json "$@" > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
r = (b.get("configs") or {}).get("rank") or {}
print("value", b["value"], "ms", b["ms_per_step"], "parity", b["parity_sample"], b.get("parity_bp"),
      "phase", b["phase_ms"], "rank", r.get("value"), r.get("parity"), "host", (b.get("host_path") or {}).get("Gbases_per_s"),
      "setup", b["setup_ms"])
PY
