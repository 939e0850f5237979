set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ingest.py tests/test_gpu_parity.py tests/test_gpu_tables.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g60.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g60.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g60.log | head -5; [ $rc = 0 ] || exit 1
for v in base prev base prev; do if [ $v = base ]; then L=kmer_spans_amd/libkmerspans.so; else L=kmer_spans_amd/libkmerspans_$v.so; fi
KS_LIB_PATH=$PWD/$L timeout -k 10 300 python tools/ab_count.py --rounds 2 --steps 3 $v: > gpurun_out/g60_$v.log 2>&1 || { tail -5 gpurun_out/g60_$v.log; exit 1; }
tail -1 gpurun_out/g60_$v.log
done
