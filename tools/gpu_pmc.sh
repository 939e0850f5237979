#!/bin/bash
# PMC passes (separate rocprofv3 runs, --pmc only with kernel records, per
# MI355X_MICROARCH.md rocprofv3 section): FETCH_SIZE, WRITE_SIZE, L2 hit/miss.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_${TAG}_fetch -o pmc --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu --out $OUT/pmc_${TAG}_bench.json "$@" > $OUT/pmc_${TAG}_fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_${TAG}_write -o pmc --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu "$@" > $OUT/pmc_${TAG}_write.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_${TAG}_l2 -o pmc --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu "$@" > $OUT/pmc_${TAG}_l2.log 2>&1
