#!/bin/bash
# scratch GPU job of the current session (see the commands below)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-job}
mkdir -p $O
cd $R
P=${2:-ab}
AB="timeout -k 10 600 python -u tools/ab_inproc.py"
if [[ $P == *a* ]]; then
$AB --rounds 3 --steps 2 --score rank one: late:KS_RESCAN_EARLY=0 --out $O/ab_rank.json > $O/ab_rank.txt 2>&1 || { tail -30 $O/ab_rank.txt; exit 1; }
tail -4 $O/ab_rank.txt
$AB --rounds 3 --steps 3 one: --out $O/ab_log2.json > $O/ab_log2.txt 2>&1 || { tail -30 $O/ab_log2.txt; exit 1; }
tail -4 $O/ab_log2.txt
$AB --rounds 3 --steps 3 --shard-of 8 one: --out $O/ab_shard8.json > $O/ab_shard8.txt 2>&1 || { tail -30 $O/ab_shard8.txt; exit 1; }
tail -4 $O/ab_shard8.txt
fi
if [[ $P == *b* ]]; then
$AB --rounds 2 --steps 2 --k 15 --score rank one: nosumm:KS_F64_P1SUMM=0 --out $O/ab_k15rank.json > $O/ab_k15rank.txt 2>&1 || { tail -30 $O/ab_k15rank.txt; exit 1; }
tail -3 $O/ab_k15rank.txt
$AB --rounds 2 --steps 3 --k 15 --score log2 one: --out $O/ab_k15log2.json > $O/ab_k15log2.txt 2>&1 || { tail -30 $O/ab_k15log2.txt; exit 1; }
tail -2 $O/ab_k15log2.txt
$AB --rounds 3 --steps 3 --k 7 --score pm1 summ: old:KS_LDS_P1SUMM=0 --out $O/ab_k7pm1.json > $O/ab_k7pm1.txt 2>&1 || { tail -30 $O/ab_k7pm1.txt; exit 1; }
tail -3 $O/ab_k7pm1.txt
$AB --rounds 3 --steps 3 --k 7 --score log2 summ: old:KS_LDS_P1SUMM=0 --out $O/ab_k7log2.json > $O/ab_k7log2.txt 2>&1 || { tail -30 $O/ab_k7log2.txt; exit 1; }
tail -3 $O/ab_k7log2.txt
KS_DEBUG_CARRY=1 timeout -k 10 300 python -u tools/ab_inproc.py --rounds 1 --steps 1 --score rank dbg: > $O/rank_debug.txt 2>&1 || { tail -30 $O/rank_debug.txt; exit 1; }
grep -E "^\[(carry|rescan|p1summ|replay)" $O/rank_debug.txt | head -12
fi
if [[ $P == *g* ]]; then
B="timeout -k 10 600 python -u bench.py --mode genomes --genomes-per-rank 4"
$B --no-cpu --out $O/genomes_pipe32.json > $O/genomes_pipe32.log 2>&1 || { tail -30 $O/genomes_pipe32.log; exit 1; }
$B --no-cpu --ext-max-gib 64 --out $O/genomes_pipe64.json > $O/genomes_pipe64.log 2>&1 || { tail -30 $O/genomes_pipe64.log; exit 1; }
$B --no-cpu --genomes-serial --out $O/genomes_serial32.json > $O/genomes_serial32.log 2>&1 || { tail -30 $O/genomes_serial32.log; exit 1; }
python3 -c "
import json
for n in ('genomes_pipe32','genomes_pipe64','genomes_serial32'):
    b=json.load(open('$O/'+n+'.json')); print(n, b['value'], b['ms_per_step'], b.get('parity_sample'))
"
fi
if [[ $P == *p* ]]; then
timeout -k 10 300 python -u tools/genome_phases.py --ext-gib 32 > $O/phases32.txt 2>&1 || { tail -30 $O/phases32.txt; exit 1; }
tail -1 $O/phases32.txt
timeout -k 10 300 python -u tools/genome_phases.py --ext-gib 140 > $O/phases140.txt 2>&1 || { tail -30 $O/phases140.txt; exit 1; }
tail -1 $O/phases140.txt
$AB --rounds 2 --steps 2 --k 15 --score rank one: --out $O/ab_k15rank.json > $O/ab_k15rank.txt 2>&1 || { tail -30 $O/ab_k15rank.txt; exit 1; }
tail -2 $O/ab_k15rank.txt
fi
if [[ $P == *x* ]]; then
$AB --rounds 3 --steps 3 --k 7 --score pm1 one: split:KS_EXACT_SPLIT=1 --out $O/ab_k7pm1_exact.json > $O/ab_k7pm1_exact.txt 2>&1 || { tail -30 $O/ab_k7pm1_exact.txt; exit 1; }
tail -2 $O/ab_k7pm1_exact.txt
$AB --rounds 3 --steps 3 --score pm1 one: split:KS_EXACT_SPLIT=1 --out $O/ab_pm1_exact.json > $O/ab_pm1_exact.txt 2>&1 || { tail -30 $O/ab_pm1_exact.txt; exit 1; }
tail -2 $O/ab_pm1_exact.txt
$AB --rounds 4 --steps 3 one: shfl:KS_NEV_SHFL=1 --out $O/ab_log2.json > $O/ab_log2.txt 2>&1 || { tail -30 $O/ab_log2.txt; exit 1; }
tail -2 $O/ab_log2.txt
fi
if [[ $P == *r* ]]; then
$AB --rounds 3 --steps 2 --score rank one: late:KS_RESCAN_EARLY=0 --out $O/ab_rank.json > $O/ab_rank.txt 2>&1 || { tail -30 $O/ab_rank.txt; exit 1; }
tail -2 $O/ab_rank.txt
$AB --rounds 2 --steps 2 --k 15 --score rank one: late:KS_RESCAN_EARLY=0 --out $O/ab_k15rank.json > $O/ab_k15rank.txt 2>&1 || { tail -30 $O/ab_k15rank.txt; exit 1; }
tail -2 $O/ab_k15rank.txt
$AB --rounds 3 --steps 3 --k 7 --score pm1 one: fp64:KS_NO_LDS_INT=1 --out $O/ab_k7pm1.json > $O/ab_k7pm1.txt 2>&1 || { tail -30 $O/ab_k7pm1.txt; exit 1; }
tail -1 $O/ab_k7pm1.txt
fi
if [[ $P == *k* ]]; then
M="timeout -k 10 300 python -u bench.py --no-cpu --no-rank --no-host-path --no-visits --steps 20"
for i in 1 2; do
$M --out $O/k8_$i.json > $O/k8_$i.log 2>&1 || { tail -20 $O/k8_$i.log; exit 1; }
KS_APPROX_K=7 $M --out $O/k7_$i.json > $O/k7_$i.log 2>&1 || { tail -20 $O/k7_$i.log; exit 1; }
done
for f in k8_1 k7_1 k8_2 k7_2; do python3 -c "import json;b=json.load(open('$O/$f.json'));print('$f', b['value'], b['ms_per_step'], b['phase_ms'])"; done
fi
