#!/bin/bash
# Session-3: expanded-table build, 8 vs 16 pairs per trip (12-bit), and the
# FP64 (weighted-rank, J = 4) build with 1 / 4 / 8 halves per trip.
set -e
O=gpurun_out/s3e
mkdir -p $O
timeout -k 10 300 python tools/ab_table.py --rounds 3 u8: u16:KS_EXT_U16=1 > $O/ab_table_c12.txt 2>&1
timeout -k 10 400 python tools/ab_table.py --rounds 3 --score rank f1: f4:KS_EXT_F64_U4=1 f8:KS_EXT_F64_U8=1 > $O/ab_table_f64.txt 2>&1
