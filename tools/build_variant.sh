#!/bin/bash
# Build an alternative libkmerspans_<name>.so for A/B runs on one GPU box
# (tools/p1_variants.sh, KS_LIB_PATH): the csrc tree of git revision REV
# ("work" = the working tree) with extra compiler flags.
# Usage: tools/build_variant.sh NAME REV [EXTRA_FLAGS...]
set -e
NAME=$1; REV=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/ksvar_XXXX)
mkdir -p $T/kmer_spans_amd/csrc $T/include
if [ "$REV" = work ]; then
  cp $R/kmer_spans_amd/csrc/*.hip $R/kmer_spans_amd/csrc/*.cpp $R/kmer_spans_amd/csrc/*.h $R/kmer_spans_amd/csrc/Makefile $T/kmer_spans_amd/csrc/
  cp $R/include/*.h $T/include/
else
  (cd $R && git archive $REV kmer_spans_amd/csrc include) | tar -x -C $T
fi
make -s -j8 -C $T/kmer_spans_amd/csrc EXTRA="$*" OUT=$R/kmer_spans_amd/libkmerspans_$NAME.so
rm -rf $T
echo built kmer_spans_amd/libkmerspans_$NAME.so
