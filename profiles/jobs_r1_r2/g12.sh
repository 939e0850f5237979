set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke12.log 2>&1 || { tail -20 gpurun_out/smoke12.log; exit 1; }
tail -1 gpurun_out/smoke12.log
timeout -k 10 400 python bench.py --gpus 2 --scale 0.05 --steps 3 --out gpurun_out/b12_g2.json > gpurun_out/b12_g2.log 2>&1 || { tail -30 gpurun_out/b12_g2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b12_g2.json')); print('gpus2', d['n_gpus'], d['value'], d['ms_per_step'], d['regions'])"
timeout -k 10 400 python bench.py --gpus 2 --mode shard --scale 0.05 --steps 3 --out gpurun_out/b12_shard.json > gpurun_out/b12_shard.log 2>&1 || { tail -30 gpurun_out/b12_shard.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b12_shard.json')); print('shard', d['n_gpus'], d['value'], d.get('merged_regions'), d.get('merged_order_ok'))"
timeout -k 10 600 python bench.py --mode genomes --genomes-per-rank 3 --out gpurun_out/b12_genomes.json > gpurun_out/b12_genomes.log 2>&1 || { tail -30 gpurun_out/b12_genomes.log; exit 1; }
cat gpurun_out/b12_genomes.json
