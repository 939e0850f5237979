set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g6.log 2>&1 || { tail -40 gpurun_out/pytest_g6.log; exit 1; }
tail -1 gpurun_out/pytest_g6.log
KS_DEBUG_CARRY=1 timeout -k 10 300 python bench.py --steps 2 --no-cpu --out gpurun_out/b6_dbg.json > gpurun_out/b6_dbg.log 2>&1 || { tail -30 gpurun_out/b6_dbg.log; exit 1; }
grep -E "p1summ|\[carry\] windows" gpurun_out/b6_dbg.log | tail -4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof6 -o run -- python3 bench.py --steps 3 --no-cpu --out gpurun_out/b6.json > gpurun_out/b6_prof.log 2>&1 || { tail -30 gpurun_out/b6_prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b6.json')); print('summ', d['value'], d['ms_per_step'], d['phase_ms'])"
f=$(find gpurun_out/prof6 -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/kernel_stats_6.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_stats_6.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["AverageNs"])/1e6:9.3f} ms x{r["Calls"]:>4}  {r["Name"][:110]}')
PY
