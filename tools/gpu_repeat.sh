#!/bin/bash
# The whole GPU suite N times in a row (no -x): how often the intermittent
# host-entry parity failure shows, with its diagnostics.
# Usage: tools/gpu_repeat.sh TAG [N]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-repeat}
N=${2:-3}
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite_$i.txt 2>&1
  rc=$?
  echo "run $i rc $rc $(tail -1 $O/suite_$i.txt)"
  grep -h "random case mismatch\|^FAILED" $O/suite_$i.txt | cut -c1-300 | head -6
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
