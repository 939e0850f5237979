set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_g37.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_g37.log; grep -E "^E  |^FAILED" gpurun_out/pytest_g37.log | head -5; [ $rc = 0 ] || exit 1
for v in c p; do if [ $v = p ]; then E=KS_NO_CONTIG_EXT=1; else E=X=1; fi; env $E timeout -k 10 300 python bench.py --score rank --steps 3 --no-cpu --out gpurun_out/g37_$v.json > gpurun_out/g37_$v.log 2>&1 || exit 1; python3 -c "import json; d=json.load(open(\"gpurun_out/g37_$v.json\")); s=d[\"setup_ms\"]; print(\"$v\", d[\"value\"], d[\"phase_ms\"][\"scan\"], s[\"table_ext_build\"], s[\"table_first_call\"], d[\"end_to_end\"][\"ms\"])"; done
