set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g10.log 2>&1 || { tail -30 gpurun_out/pytest_g10.log; exit 1; }
tail -1 gpurun_out/pytest_g10.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof10 -o run -- python3 bench.py --steps 5 --no-cpu --out gpurun_out/b10.json > gpurun_out/b10_prof.log 2>&1 || { tail -30 gpurun_out/b10_prof.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b10.json')); print('bench', d['value'], d['ms_per_step'], d['phase_ms'])"
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/prof10/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    if r["Name"].startswith("void at::") or "rocclr" in r["Name"]: continue
    print(f'{float(r["AverageNs"])/1e6:9.3f} ms x{r["Calls"]:>4}  {r["Name"][:100]}')
PY
