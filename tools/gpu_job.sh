#!/bin/bash
# In-process A/B runs of this round's switches (tools/ab_inproc.py: all
# variants on the same allocations).  Usage: tools/gpu_job.sh TAG [PARTS]
#   m: metric (log2 k = 13)   r: weighted rank k = 13 / 15   x: +-1 k = 7 / 13
#   p: per-genome phases (config 5)   d: rank carry / rescan diagnostics
#   s: shard-of-8 and config 2 (fixed cost at small sizes)   q: predictor sampling stride
#   c: GPU tests, then pass-1 summaries read in place vs copied   f: split fraction (metric)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-job}
P=${2:-mrx}
mkdir -p $O
cd $R
AB="timeout -k 10 600 python -u tools/ab_inproc.py"
ab() { name=$1; shift; $AB "$@" --out $O/$name.json > $O/$name.txt 2>&1 || { tail -30 $O/$name.txt; exit 1; }; grep -v "^round\|amdgpu.ids" $O/$name.txt | cut -c1-300; }
if [[ $P == *m* ]]; then
ab ab_log2 --rounds 3 --steps 3 one: approx8:KS_APPROX_K=8
fi
if [[ $P == *r* ]]; then
ab ab_rank --rounds 3 --steps 2 --score rank one: late:KS_RESCAN_EARLY=0 summ:KS_F64_P1SUMM=1
ab ab_k15rank --rounds 2 --steps 2 --k 15 --score rank one: late:KS_RESCAN_EARLY=0
fi
if [[ $P == *x* ]]; then
ab ab_k7pm1 --rounds 3 --steps 3 --k 7 --score pm1 one: fp64:KS_NO_LDS_INT=1 gen:KS_NO_EXACT=1
ab ab_pm1 --rounds 3 --steps 3 --score pm1 one: gen:KS_NO_EXACT=1
fi
if [[ $P == *s* ]]; then
ab ab_shard8 --rounds 4 --steps 10 --shard-of 8 one: late:KS_RESCAN_EARLY=0 f60:KS_SPLIT_FRAC=0.6 f80:KS_SPLIT_FRAC=0.8
ab ab_cfg2 --rounds 4 --steps 10 --k 11 --ncontigs 1 one: late:KS_RESCAN_EARLY=0 f80:KS_SPLIT_FRAC=0.8
fi
if [[ $P == *q* ]]; then
ab ab_pred_log2 --rounds 3 --steps 3 one: ps4:KS_PRED_PS=4 ps8:KS_PRED_PS=8
ab ab_pred_shard8 --rounds 4 --steps 10 --shard-of 8 one: ps4:KS_PRED_PS=4
fi
if [[ $P == *c* ]]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
ab ab_sel_log2 --rounds 3 --steps 3 one: copy:KS_SUMM_COPY=1
ab ab_sel_shard8 --rounds 4 --steps 10 --shard-of 8 one: copy:KS_SUMM_COPY=1
ab ab_sel_k15 --rounds 2 --steps 2 --k 15 one: copy:KS_SUMM_COPY=1
fi
if [[ $P == *f* ]]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
ab ab_frac_log2 --rounds 3 --steps 3 one: f70:KS_SPLIT_FRAC=0.7 f55:KS_SPLIT_FRAC=0.55 f65:KS_SPLIT_FRAC=0.65
ab ab_frac_rank --rounds 3 --steps 2 --score rank one: f70:KS_SPLIT_FRAC=0.7
ab ab_frac_k15 --rounds 2 --steps 2 --k 15 one: f70:KS_SPLIT_FRAC=0.7
ab ab_frac_k15rank --rounds 2 --steps 2 --k 15 --score rank one: f70:KS_SPLIT_FRAC=0.7
fi
if [[ $P == *p* ]]; then
timeout -k 10 300 python -u tools/genome_phases.py --ext-gib 32 > $O/phases32.txt 2>&1 || { tail -30 $O/phases32.txt; exit 1; }
tail -1 $O/phases32.txt
fi
if [[ $P == *d* ]]; then
KS_DEBUG_CARRY=1 timeout -k 10 300 python -u tools/ab_inproc.py --rounds 1 --steps 1 --score rank dbg: > $O/rank_debug.txt 2>&1 || { tail -30 $O/rank_debug.txt; exit 1; }
grep -E "^\[(carry|rescan|p1summ|replay)" $O/rank_debug.txt | head -12
fi
