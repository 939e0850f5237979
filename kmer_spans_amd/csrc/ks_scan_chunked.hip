// ks_scan_chunked.hip -- chunked carry scan (algo 1).  Placeholder until the
// chunked implementation lands; dispatch never selects it automatically yet.
#include "ks_scan_common.h"

namespace ks {
ks_status scan_chunked(ks_ctx *, const ks_dev_seqs *, const Runs &, int, const TableView &, uint64_t,
                       double, uint32_t *, const RegionBuf &, ks_scan_stats *) {
  return fail(KS_ERR_INTERNAL, "chunked scan not available in this build");
}
}  // namespace ks
