set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
bash tools/gpu_r2.sh r2d || exit 1
tools/ab_bench.sh ns2 "--steps 3 --no-cpu" base nostore || exit 1
