#!/bin/bash
# Multi-rank rehearsals on the one GPU of a box (gloo: two ranks share the
# card; the 8-GPU RCCL runs are the driver's): shard mode (records gathered,
# merged, parity) and config 5 (genomes per rank).  Usage: tools/gpu_multi.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-multi}
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --gpus 2 --scale 0.05 --steps 3 --out $O/shard2.json > $O/shard2.log 2>&1 || { tail -30 $O/shard2.log; exit 1; }
python3 -c "import json;b=json.load(open('$O/shard2.json'));print('shard2', b['value'], b['ms_per_step'], b.get('parity_sample'), b.get('merged_order_ok'), b.get('gather_ms'), b['config'].get('parallelism'))"
timeout -k 10 300 python bench.py --gpus 2 --scale 0.05 --mode genomes --genomes-per-rank 2 --out $O/genomes2.json > $O/genomes2.log 2>&1 || { tail -30 $O/genomes2.log; exit 1; }
python3 -c "import json;b=json.load(open('$O/genomes2.json'));print('genomes2', b['value'], b['ms_per_step'], b.get('parity_sample'), b['config'].get('parallelism'))"
