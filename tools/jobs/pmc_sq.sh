#!/bin/bash
# SQ instruction / busy counters of the metric step (is pass 1 VALU-bound?).  Usage: tools/jobs/pmc_sq.sh TAG
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" $O/avail.txt | sort -u > $O/sq_names.txt || true
B="python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-rank --no-visits --no-host-path"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD -d $O/p1 -o pmc --output-format csv -- $B > $O/p1.log 2>&1 || { tail -5 $O/p1.log; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -d $O/p2 -o pmc --output-format csv -- $B > $O/p2.log 2>&1 || { tail -5 $O/p2.log; }
for p in p1 p2; do
  f=$(find $O/$p -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    n = r.get("Kernel_Name", "")
    if "k_pass1l" in n or "k_pass1p" in n:
        agg[n[:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for n, cs in agg.items():
    print(n)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {v:.4g}")
PY
done
