#!/bin/bash
# Register / scratch / occupancy of the library's kernels (compile-time remarks).
# Usage: tools/kres.sh kmer_spans_amd/csrc/ks_scan_chunked.hip
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -c "$f" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -v rocprim |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed 's/.*remark: *//; s/ \[-Rpass.*//' |
  paste - - - - | grep "_ZN2ks" | sed 's/Function Name: _ZN2ks12_GLOBAL__N_1//' | awk '{print}' | cut -c1-160
