#!/bin/bash
# Session-3: expanded-table build variants (pairs per trip, store policy).
set -e
O=gpurun_out/s3d
mkdir -p $O
timeout -k 10 300 python tools/ab_table.py --rounds 4 u4: u8:KS_EXT_U8=1 plain:KS_EXT_PLAIN=1 u1:KS_EXT_U1=1 > $O/ab_table.txt 2>&1
