#!/bin/bash
# SQ occupancy / wait counters of one bench line's kernels (one --pmc pass).
# Usage: tools/gpu_sqpmc.sh TAG "bench args"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
A="$2 --no-cpu --no-rank --no-host-path --no-visits --parity none"
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/sq -o sq --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $A --out $O/sq_bench.json > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
F=$(find $O/sq -name '*counter_collection.csv' | head -1)
python3 - "$F" > $O/sq_summary.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in rows:
    name = r.get("Kernel_Name", "")
    short = name.split("(")[0].split("::")[-1][:40]
    agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))[:25]:
    w = v.get("SQ_WAVES", 0) or 1
    print(f"{k:40s} gui {v.get('GRBM_GUI_ACTIVE',0):12.0f} waves {v.get('SQ_WAVES',0):10.0f} "
          f"wave_cyc/wave {v.get('SQ_WAVE_CYCLES',0)/w:10.0f} busy {v.get('SQ_BUSY_CYCLES',0):12.0f} "
          f"wait_inst/wave_cyc {v.get('SQ_WAIT_INST_ANY',0)/max(1,v.get('SQ_WAVE_CYCLES',0)):.3f} "
          f"wait_any/wave_cyc {v.get('SQ_WAIT_ANY',0)/max(1,v.get('SQ_WAVE_CYCLES',0)):.3f} "
          f"valu/wave {v.get('SQ_INSTS_VALU',0)/w:8.0f} vmem/wave {v.get('SQ_INSTS_VMEM_RD',0)/w:8.0f}")
PY
cat $O/sq_summary.txt
