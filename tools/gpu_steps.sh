#!/bin/bash
# Run named GPU steps in order, each under its own time limit, output under
# gpurun_out/<tag>/<step>.txt; stop at the first step that ends with anything
# but 0 or 1 (a fault, an abort, a time limit).  Usage:
#   tools/gpu_steps.sh TAG "name|seconds|command" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 $secs bash -c "$cmd" > $O/$name.txt 2>&1
  rc=$?
  echo "== $name rc $rc: $(tail -1 $O/$name.txt | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
done
