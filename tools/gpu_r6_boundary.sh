set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6a
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_rccl.py tests/test_multi.py tests/test_gpu_ctx_guard.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -12 $O/pytest.log
timeout -k 10 300 python tools/probes/free_order_probe.py --out $O/free_order.json > $O/free_order.log 2>&1 || { tail -30 $O/free_order.log; exit 1; }
python -c "import json;d=json.load(open('$O/free_order.json'));[print(v['variant'],v['results_equal_oracle'],v['min_drain_plus_free_ms'],[(f['where'],round(f['drain_ms'],1),round(f['hipfree_ms'],1)) for f in v['frees']][:6]) for v in d['variants']]"
