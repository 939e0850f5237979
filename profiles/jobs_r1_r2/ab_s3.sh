#!/bin/bash
# Round-2 session-3 A/B on one GPU box: count kernels (next-tile prefetch in
# the partition passes, 4 loads in flight in k_bins) against the HEAD build
# (libkmerspans_base.so via KS_LIB_PATH, alternating processes), and the
# run pass's prefetched byte before each unit (in process, KS_NEV_LATE_PREV).
set -e
O=gpurun_out/s3ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "count or ingest or visit or multi" > $O/pytest_count.txt 2>&1
for i in 1 2; do
  KS_LIB_PATH=$PWD/kmer_spans_amd/libkmerspans_base.so timeout -k 10 200 python tools/ab_count.py --k 13 base: \
    > $O/count_base_$i.txt 2>&1
  timeout -k 10 200 python tools/ab_count.py --k 13 new: > $O/count_new_$i.txt 2>&1
done
timeout -k 10 200 python tools/ab_count.py --k 15 new: > $O/count_new_k15.txt 2>&1
timeout -k 10 300 python tools/ab_inproc.py --rounds 4 --steps 3 pre: late:KS_NEV_LATE_PREV=1 > $O/ab_nev.txt 2>&1
