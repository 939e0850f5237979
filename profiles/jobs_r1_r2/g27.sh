set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_smallk.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g27.log 2>&1; rc=$?; grep -E "^E  |^FAILED|passed|failed" gpurun_out/pytest_g27.log | tail -6; [ $rc = 0 ] || exit 1
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt27 -o kt --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --out $R/gpurun_out/kt27_bench.json > $R/gpurun_out/kt27.log 2>&1) || exit 1
timeout -k 10 400 python tools/ab_inproc.py --rounds 3 --steps 3 new: noov:KS_NO_P0_OVERLAP=1 --out gpurun_out/ab_g27.json
