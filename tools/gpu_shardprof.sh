#!/bin/bash
# Kernel trace + step timeline of the 8-way shard step (bench.py --shard-of 8:
# the largest of eight LPT shards of the metric genome, the whole genome's
# table) with the given environment.  Usage: tools/gpu_shardprof.sh TAG [N] "ENV=V ..."
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
N=${2:-8}
mkdir -p $O
for kv in $3; do export $kv; done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --shard-of $N --steps 3 --warmup 1 --no-cpu --no-rank --no-host-path --no-visits --out $O/bench.json > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
F=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $F > $O/step_timeline.txt || true
cat $O/step_timeline.txt | tail -90
python3 -c "import json;b=json.load(open('$O/bench.json'));print(b['ms_per_step'],b['phase_ms'])"
