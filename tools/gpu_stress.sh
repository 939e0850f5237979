#!/bin/bash
# tools/stress_config1.py under each path switch (one process each).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-stress}
mkdir -p $O
cd $R
run() { tag=$1; shift; env "$@" timeout -k 10 240 python -u tools/stress_config1.py 40 > $O/$tag.txt 2>&1; rc=$?; echo "$tag rc $rc"; grep -v amdgpu $O/$tag.txt | tail -4 | cut -c1-300; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run base KS_X=0
run base2 KS_X=0
run noexact KS_NO_EXACT=1
run nolint KS_NO_LDS_INT=1
run noldstab KS_NO_LDS_TABLE=1
run cache KS_HOST_CACHE=1
