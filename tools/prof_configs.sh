set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_rank -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --score rank --out $OUT/rank.json > $OUT/prof_rank.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_k15 -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu --k 15 --out $OUT/k15.json > $OUT/prof_k15.log 2>&1 || exit 1
cat $OUT/rank.json $OUT/k15.json
