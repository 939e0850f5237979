#!/bin/bash
# 2-rank shard rehearsal (gloo, both ranks on the one GPU) and the 8-way
# shard fixed cost on one GPU.  Usage: tools/jobs/multi.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --gpus 2 --scale 0.05 --steps 3 --no-rank --no-host-path --no-visits \
  --out $O/shard2.json > $O/shard2.log 2>&1 || { tail -30 $O/shard2.log; exit 1; }
python -c "import json;b=json.load(open('$O/shard2.json'));print('shard2', b['value'], b.get('merged_order_ok'), b.get('parity_sample'), b.get('parity_bp'), b['config'])"
for S in 8 4 2; do
timeout -k 10 400 python bench.py --shard-of $S --steps 10 --no-cpu --no-rank --no-host-path --no-visits \
  --out $O/shardof$S.json > $O/shardof$S.log 2>&1 || { tail -30 $O/shardof$S.log; exit 1; }
python -c "import json;b=json.load(open('$O/shardof$S.json'));print('shard-of $S', b['value'], b['ms_per_step'], b['phase_ms'], b['roofline']['achieved'], b.get('config'))"
done
