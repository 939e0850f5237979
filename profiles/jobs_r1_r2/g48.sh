set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g48.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g48.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g48.log | head -5; [ $rc = 0 ] || exit 1
timeout -k 10 400 python bench.py --gpus 2 --scale 0.05 --steps 3 --out gpurun_out/b48_g2.json > gpurun_out/b48_g2.log 2>&1 || { tail -30 gpurun_out/b48_g2.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b48_g2.json')); print('genome x2', d['n_gpus'], d['value'], d['parity_sample'])"
timeout -k 10 400 python bench.py --gpus 2 --mode shard --scale 0.05 --steps 3 --out gpurun_out/b48_shard.json > gpurun_out/b48_shard.log 2>&1 || { tail -30 gpurun_out/b48_shard.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b48_shard.json')); print('shard x2', d['n_gpus'], d['value'], d['parity_sample'])"
timeout -k 10 400 python bench.py --mode genomes --scale 0.05 --steps 2 --out gpurun_out/b48_genomes.json > gpurun_out/b48_genomes.log 2>&1 || { tail -30 gpurun_out/b48_genomes.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b48_genomes.json')); print('genomes', d['n_gpus'], d['value'], d.get('parity_sample'))"
