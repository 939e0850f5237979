#!/bin/bash
# Session-3 final: the final-build evidence (tools/s3_final.sh), then the
# expanded-table build A/Bs of the FP64 (weighted rank, J = 4) and uint16
# (J = 4, host entry / genomes mode) builds: 8 per trip (default) vs 1 / 4.
set -e
bash tools/s3_final.sh s3h
O=gpurun_out/s3h
timeout -k 10 400 python tools/ab_table.py --rounds 3 --score rank f8: f1:KS_EXT_U1=1 f4:KS_EXT_F64_U4=1 > $O/ab_table_f64.txt 2>&1
timeout -k 10 300 python tools/ab_table.py --rounds 3 --ext-max-gib 32 u8: u1:KS_EXT_U1=1 > $O/ab_table_u16.txt 2>&1
