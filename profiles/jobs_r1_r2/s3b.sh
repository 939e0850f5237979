#!/bin/bash
# Session-3 check: full GPU suite with the concurrent visit count, then the
# bench with it and with KS_VISITS_SERIAL=1 (the count after the scan).
set -e
O=gpurun_out/s3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu > $O/bench_conc.json 2> $O/bench_conc.err
KS_VISITS_SERIAL=1 timeout -k 10 300 python bench.py --no-cpu > $O/bench_serial.json 2> $O/bench_serial.err
