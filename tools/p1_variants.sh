#!/bin/bash
# Pass-1 kernel variants (alternative builds of libkmerspans.so selected with
# KS_LIB_PATH): bench ms of k_pass1p + one FETCH_SIZE PMC pass each.
# Usage: tools/p1_variants.sh TAG variant...   (variant = suffix of libkmerspans_<v>.so, "base" = default)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = base ]; then lib=$R/kmer_spans_amd/libkmerspans.so; else lib=$R/kmer_spans_amd/libkmerspans_$v.so; fi
  cd $R
  KS_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --out $OUT/var_${TAG}_$v.json > $OUT/var_${TAG}_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/var_${TAG}_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/var_${TAG}_$v.json')); print('$v', d['value'], d['phase_ms'])"
  cd /tmp
  KS_LIB_PATH=$lib timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/var_${TAG}_${v}_fetch -o pmc --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/var_${TAG}_${v}_fetch.log 2>&1 || { echo "pmc $v failed"; tail -20 $OUT/var_${TAG}_${v}_fetch.log; exit 1; }
  python3 - <<PY
import csv, glob
for f in glob.glob('$OUT/var_${TAG}_${v}_fetch/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'pass1' in r['Kernel_Name']:
            print('$v', r['Kernel_Name'][:40], r['Counter_Name'], r['Counter_Value'])
PY
done
