set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g59.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g59.log; [ $rc = 0 ] || exit 1
for v in base prev base prev; do if [ $v = base ]; then L=kmer_spans_amd/libkmerspans.so; else L=kmer_spans_amd/libkmerspans_$v.so; fi
KS_LIB_PATH=$PWD/$L KS_DEBUG_CARRY=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu --out gpurun_out/g59_$v.json > gpurun_out/g59_$v.log 2>&1 || exit 1
KS_LIB_PATH=$PWD/$L timeout -k 10 300 python tools/ab_inproc.py --rounds 2 --steps 3 x: --out gpurun_out/g59i_$v.json > gpurun_out/g59i_$v.log 2>&1 || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/g59i_$v.json'))['x']; print('$v', d['min_ms'], d['best_phases']['ms_layout'])"; grep "p1summ\]" gpurun_out/g59_$v.log | head -1
done
