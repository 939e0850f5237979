#!/bin/bash
# SQ / LDS / TCC counters of the k-mer count kernels (one in-process count of the metric genome per pass).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- python3 $R/tools/ab_count.py --rounds 1 --steps 2 "$@" > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
find $O/stats -name '*kernel_stats.csv' | head -1 | xargs -I{} sh -c 'grep -E "k_part|k_bins|k_bucket" {} | cut -c1-200'
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS" "WRITE_SIZE GRBM_GUI_ACTIVE" "FETCH_SIZE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $O/pmc$i -o pmc --output-format csv -- python3 $R/tools/ab_count.py --rounds 1 --steps 1 "$@" > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
done
cd $R
python3 - $O <<'PY'
import glob, sys
sys.path.insert(0, "tools")
from pmc_summary import load
o = sys.argv[1]
agg = {}
for f in glob.glob(o + "/pmc*/**/*counter_collection.csv", recursive=True):
    for n, cs in load(f).items():
        if not any(s in n for s in ("k_part", "k_bins", "k_bucket", "k_count")): continue
        for c, vals in cs.items(): agg.setdefault(n, {})[c] = sum(vals)
for n, d in agg.items():
    print(n)
    for c, v in sorted(d.items()): print(f"   {c:24s} {v:18.1f}")
PY
