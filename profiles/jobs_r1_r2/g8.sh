set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "code12" > gpurun_out/pytest_g8_$i.log 2>&1; echo "rc=$?"; grep -E "passed|failed|AssertionError" gpurun_out/pytest_g8_$i.log | head -5
done
KS_NO_P1_SUMMARY=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "code12" > gpurun_out/pytest_g8_ns.log 2>&1; echo "rc(no summ)=$?"; grep -E "passed|failed|AssertionError" gpurun_out/pytest_g8_ns.log | head -5
