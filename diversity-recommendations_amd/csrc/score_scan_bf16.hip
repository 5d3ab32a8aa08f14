// bf16-table instantiations of the score scan (score_scan.h): row widths
// d = 32, 64, 128, 256, 512 (W = d).
#include "score_scan.h"

namespace dr_topk {

bool launch_scan_bf16(const Plan& p, const TopkArgs& a, int w, bool seeded, hipStream_t s) {
  return launch_scan_widths<false, 32, 64, 128, 256, 512>(p, a, w, seeded, s);
}

}  // namespace dr_topk
