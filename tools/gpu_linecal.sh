#!/bin/bash
# HBM-byte calibration of random line reads (MI355X_MICROARCH.md: calibrate
# FETCH_SIZE on a known byte count of your own access pattern): the coalesced
# group forms of tools/probes/line_bench.hip under rocprofv3 --pmc FETCH_SIZE
# (128 GiB table), then the rates from a 128 MiB table (Infinity-Cache
# resident) and a 1 GiB table.  Usage: tools/gpu_linecal.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc -o pmc --output-format csv -- $R/tools/probes/line_bench 131072 group > $O/pmc_run.txt 2>&1 || { tail -20 $O/pmc_run.txt; exit 1; }
grep '^{' $O/pmc_run.txt
timeout -k 10 300 $R/tools/probes/line_bench 128 group > $O/mall.txt 2>&1 || { tail -20 $O/mall.txt; exit 1; }
cat $O/mall.txt
timeout -k 10 300 $R/tools/probes/line_bench 1024 group > $O/gib1.txt 2>&1 || { tail -20 $O/gib1.txt; exit 1; }
cat $O/gib1.txt
F=$(find $O/pmc -name '*counter_collection.csv' | head -1)
python3 - "$F" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.OrderedDict()
for r in rows:
    key = (r.get("Kernel_Name") or r.get("Kernel-Name"))[:60]
    agg.setdefault(key, []).append(float(r.get("Counter_Value") or r.get("Counter-Value")))
for k, v in agg.items():
    print(f"{k:60s} dispatches {len(v)} FETCH_SIZE_KB per dispatch {sum(v)/len(v):.0f} -> bytes per line read {sum(v)/len(v)*1024/2**31:.1f}")
PY
