// ks_version.cpp -- ks_version(): the library name plus a build id, a hash of
// every source of the library and of the build flags (Makefile), so that
// measurements taken on one build (rocprofv3 PMC summaries under profiles/)
// can be matched to the library that bench.py loads.
#include "../../include/kmer_spans.h"

#ifndef KS_BUILD_ID
#define KS_BUILD_ID "unknown"
#endif

extern "C" const char *ks_version(void) { return "kmer_spans_amd 0.2 gfx950 build " KS_BUILD_ID; }
