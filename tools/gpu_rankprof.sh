#!/bin/bash
# Kernel trace + step timeline and the HBM traffic (FETCH_SIZE, WRITE_SIZE in
# passes of their own) of one bench line.  Usage:
#   tools/gpu_rankprof.sh TAG "bench args"
# e.g. tools/gpu_rankprof.sh r5rank13 "--score rank --k 13"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
A="$2 --no-cpu --no-rank --no-host-path --no-visits --parity none"
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $A --out $O/prof_bench.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/step_timeline.txt || true
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $A --out $O/pmc_bench.json > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 $A > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
cd $R
python3 tools/pmc_assemble.py $O/pmc_bench.json $O/pmc_summary.json $(find $O/pmc_fetch $O/pmc_write -name '*counter_collection.csv') > $O/pmc_assemble.txt 2>&1 || { tail -20 $O/pmc_assemble.txt; exit 1; }
head -30 $O/pmc_assemble.txt
tail -1 $O/step_timeline.txt
