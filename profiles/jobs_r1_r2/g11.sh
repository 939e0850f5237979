set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in base ps2; do
  if [ $v = base ]; then L=kmer_spans_amd/libkmerspans.so; else L=kmer_spans_amd/libkmerspans_$v.so; fi
  KS_LIB_PATH=$L KS_DEBUG_CARRY=1 timeout -k 10 300 python bench.py --steps 2 --no-cpu --out gpurun_out/b11_$v.json > gpurun_out/b11_$v.log 2>&1 || { tail -20 gpurun_out/b11_$v.log; exit 1; }
  grep p1summ gpurun_out/b11_$v.log | tail -1
done
tools/ab_bench.sh g11 "--steps 5 --no-cpu" base ps2 base ps2 || exit 1
