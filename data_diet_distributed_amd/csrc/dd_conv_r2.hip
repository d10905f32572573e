// conv3x3_r2_kernel instantiations (the 16x16 / 8x8 / 4x4 tiles of the scoring passes and the
// 32x32 A/B forms); the kernel template lives in dd_conv_kern.h.
#include "dd_conv_kern.h"

namespace dd {
namespace conv {

int dispatch_r2(int w, int k, const Args& a, hipStream_t st) {
  if (w == 32 && k == 4000 + 100 + 20 + 1) return launch_r2<32, 4, 1, 2, 1>(a, st);
  if (w == 32 && k == 8000 + 100 + 10 + 2) return launch_r2<32, 8, 1, 1, 2, true>(a, st);
  if (w == 16 && k == 8000 + 100 + 10 + 4) return launch_r2<16, 8, 1, 1, 4>(a, st);
  if (w == 8 && k == 8000 + 200 + 10 + 4) return launch_r2<8, 8, 2, 1, 4>(a, st);
  if (w == 4 && k == 4000 + 800 + 10 + 4) return launch_r2<4, 4, 8, 1, 4>(a, st);
  set_error("dd_conv3x3_forward: no r2 kernel for tile key %d at w=%d", k, w);
  return DD_EINVAL;
}

}  // namespace conv
}  // namespace dd
