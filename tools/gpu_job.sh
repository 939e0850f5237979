#!/bin/bash
# scratch GPU job of the current session (see the commands below)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-job}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
V="one:KS_PARTS_FRAC=0 p55:KS_PARTS_FRAC=0.55 p65:KS_PARTS_FRAC=0.65 p75:KS_PARTS_FRAC=0.75"
timeout -k 10 900 python -u tools/ab_inproc.py --rounds 3 --steps 2 --score rank one:KS_PARTS_FRAC=0 nosumm:KS_PARTS_FRAC=0,KS_F64_P1SUMM=0 p55:KS_PARTS_FRAC=0.55 p55nosumm:KS_PARTS_FRAC=0.55,KS_F64_P1SUMM=0 p70:KS_PARTS_FRAC=0.7 --out $O/ab_rank.json > $O/ab_rank.txt 2>&1 || { tail -30 $O/ab_rank.txt; exit 1; }
tail -6 $O/ab_rank.txt
timeout -k 10 600 python -u tools/ab_inproc.py --rounds 3 --steps 3 $V --out $O/ab_log2.json > $O/ab_log2.txt 2>&1 || { tail -30 $O/ab_log2.txt; exit 1; }
tail -5 $O/ab_log2.txt
timeout -k 10 600 python -u tools/ab_inproc.py --rounds 3 --steps 3 --shard-of 8 one:KS_PARTS_FRAC=0,KS_PREDICT_BOTH_FIRST=0 bf:KS_PARTS_FRAC=0 p55:KS_PARTS_FRAC=0.55,KS_PREDICT_BOTH_FIRST=0 p55bf:KS_PARTS_FRAC=0.55 --out $O/ab_shard8.json > $O/ab_shard8.txt 2>&1 || { tail -30 $O/ab_shard8.txt; exit 1; }
tail -5 $O/ab_shard8.txt
timeout -k 10 600 python -u bench.py --mode genomes --genomes-per-rank 3 --out $O/genomes_pipe.json > $O/genomes_pipe.log 2>&1 || { tail -30 $O/genomes_pipe.log; exit 1; }
timeout -k 10 600 python -u bench.py --mode genomes --genomes-per-rank 3 --genomes-serial --no-cpu --out $O/genomes_serial.json > $O/genomes_serial.log 2>&1 || { tail -30 $O/genomes_serial.log; exit 1; }
python3 -c "
import json
for n in ('genomes_pipe','genomes_serial'):
    b=json.load(open('$O/'+n+'.json')); print(n, b['value'], b['ms_per_step'], b.get('parity_sample'))
"
timeout -k 10 600 python -u tools/ab_inproc.py --rounds 3 --steps 3 --k 7 --score pm1 summ: old:KS_LDS_P1SUMM=0 --out $O/ab_k7pm1.json > $O/ab_k7pm1.txt 2>&1 || { tail -30 $O/ab_k7pm1.txt; exit 1; }
tail -3 $O/ab_k7pm1.txt
timeout -k 10 600 python -u tools/ab_inproc.py --rounds 3 --steps 3 --k 7 --score log2 summ: old:KS_LDS_P1SUMM=0 --out $O/ab_k7log2.json > $O/ab_k7log2.txt 2>&1 || { tail -30 $O/ab_k7log2.txt; exit 1; }
tail -3 $O/ab_k7log2.txt
KS_DEBUG_CARRY=1 timeout -k 10 300 python -u tools/ab_inproc.py --rounds 1 --steps 1 --score rank dbg: > $O/rank_debug.txt 2>&1 || { tail -30 $O/rank_debug.txt; exit 1; }
grep -E "^\[(carry|rescan|p1summ|replay)" $O/rank_debug.txt | head -30
