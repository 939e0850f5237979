#!/bin/bash
# The random parity cases with every fresh workspace slot filled with one byte
# (KS_DEBUG_POISON): a read of workspace the call did not write shows up
# reproducibly.  Usage: tools/gpu_poison.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-poison}
mkdir -p $O
cd $R
for p in 0x00 0xff 0x7f 0x01 0x40 0xc0 0x3f 0x80; do
  KS_DEBUG_POISON=$p timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "random" --timeout 240 --timeout-method thread > $O/poison_$p.txt 2>&1
  rc=$?
  echo "poison $p rc $rc $(tail -1 $O/poison_$p.txt)"
  grep -h "random case mismatch\|AssertionError: ((" $O/poison_$p.txt | cut -c1-400 | head -4
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
