set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g56.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g56.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g56.log | head -5; [ $rc = 0 ] || exit 1
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt56 -o kt --output-format csv -- python $R/bench.py --steps 3 --warmup 1 --no-cpu --out $R/gpurun_out/kt56_bench.json > $R/gpurun_out/kt56.log 2>&1) || exit 1
timeout -k 10 400 python tools/ab_inproc.py --rounds 3 --steps 3 base: --out gpurun_out/ab_g56.json
