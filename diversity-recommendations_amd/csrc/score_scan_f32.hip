// fp32-table instantiations of the score scan (score_scan.h): the
// fp32-faithful scoring mode, exact fp32 fmaf chains on v_mfma_f32_32x32x2_f32.
// Row widths d = 32, 64, 128, 256 (W = 2d).
#include "score_scan.h"

namespace dr_topk {

bool launch_scan_f32(const Plan& p, const TopkArgs& a, int w, bool seeded, hipStream_t s) {
  return launch_scan_widths<true, 64, 128, 256, 512>(p, a, w, seeded, s);
}

}  // namespace dr_topk
