#!/bin/bash
# SQ counters of the count kernels (tools/ab_count.py, one k = 13 count), two
# passes of at most 8 SQ counters each; per-kernel summary to sq_summary.txt.
# Usage: tools/gpu_countsq.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
n=0
for P in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 300 rocprofv3 --pmc $P -d $O/sq$n -o sq --output-format csv -- python3 $R/tools/ab_count.py --k 13 --rounds 1 --steps 1 new: > $O/sq$n.log 2>&1 || { tail -20 $O/sq$n.log; exit 1; }
done
python3 - $O <<'PY' > $O/sq_summary.txt
import csv, sys, collections, re, glob
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r.get("Kernel_Name", ""))
        if m:
            agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:6]:
    w = v.get("SQ_WAVES", 1) / 2 or 1  # (both passes count SQ_WAVES)
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    print(k, {c: round(x / w, 1) for c, x in sorted(v.items()) if c != "SQ_WAVES"}, "| fractions of wave cycles:",
          {c: round(v.get(c, 0) / wc, 3) for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")})
PY
cat $O/sq_summary.txt
