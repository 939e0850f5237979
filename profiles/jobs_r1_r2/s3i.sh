#!/bin/bash
# Session-3: gated second passes on a small grid -- in-process A/B against the
# full grid (KS_GATED_FULL), then the final-build evidence (tools/s3_final.sh).
set -e
mkdir -p gpurun_out/s3i
timeout -k 10 300 python tools/ab_inproc.py --rounds 4 --steps 3 small: full:KS_GATED_FULL=1 > gpurun_out/s3i/ab_gated.txt 2>&1
bash tools/s3_final.sh s3i
