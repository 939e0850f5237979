"""kmer_spans_amd -- MI355X-native k-mer span scanner (drop-in for the
span-scan path of lmjakt/kmer_spans).

Public API mirrors kmer_spans.R: kmer_counts, kmer_regions,
kmer_low_comp_regions, kmer_seq; score tables log2_table, pm1_table,
rank_table.  Device-resident entry points live in kmer_spans_amd.device.
All results come from libkmerspans.so (HIP, gfx950); there is no CPU path.
"""
from ._lib import KmerSpansError, LIB_PATH, context  # noqa: F401
from .api import (kmer_counts, kmer_low_comp_regions, kmer_regions, kmer_seq,  # noqa: F401
                  kmer_magic, kmers_to_file, log2_table, lr_regions, pm1_table, rank_table, read_fasta,
                  read_kmers, set_devices, get_devices, window_kmer_dist, write_kmers)

__all__ = ["kmer_counts", "kmer_regions", "kmer_low_comp_regions", "kmer_seq", "lr_regions", "log2_table",
           "pm1_table", "rank_table", "kmer_magic", "kmers_to_file", "read_kmers", "write_kmers", "read_fasta",
           "window_kmer_dist", "set_devices", "get_devices", "KmerSpansError", "context"]
