// conv3x3_kernel instantiations of the narrow / wide tiles other than the 32x32 narrow one
// (16x16, 8x8, 4x4 fallbacks for channel counts the r2 tiles do not take, and the A/B
// families); the kernel template lives in dd_conv_kern.h.
#include "dd_conv_kern.h"

namespace dd {
namespace conv {

int dispatch_small(int w, int k, const Args& a, hipStream_t st) {
  if (w == 32) {
    if (k == 4000 + 100 + 20 + 2) return launch<32, 4, 1, 2, 2>(a, st);
    if (k == 8000 + 100 + 20 + 1) return launch<32, 8, 1, 2, 1>(a, st);
  } else if (w == 16) {
    if (k == 8000 + 100 + 20 + 2) return launch<16, 8, 1, 2, 2>(a, st);
    if (k == 16000 + 100 + 20 + 1) return launch<16, 16, 1, 2, 1>(a, st);
    if (k == 8000 + 100 + 10 + 2) return launch<16, 8, 1, 1, 2>(a, st);
  } else if (w == 8) {
    if (k == 8000 + 200 + 20 + 2) return launch<8, 8, 2, 2, 2>(a, st);
    if (k == 8000 + 400 + 20 + 1) return launch<8, 8, 4, 2, 1>(a, st);
    if (k == 8000 + 200 + 10 + 2) return launch<8, 8, 2, 1, 2>(a, st);
    if (k == 8000 + 100 + 10 + 2) return launch<8, 8, 1, 1, 2>(a, st);
  } else if (w == 4) {
    if (k == 4000 + 800 + 20 + 2) return launch<4, 4, 8, 2, 2>(a, st);
    if (k == 4000 + 1600 + 20 + 1) return launch<4, 4, 16, 2, 1>(a, st);
    if (k == 4000 + 400 + 10 + 2) return launch<4, 4, 4, 1, 2>(a, st);
  }
  set_error("dd_conv3x3_forward: no kernel for tile key %d at w=%d", k, w);
  return DD_EINVAL;
}

}  // namespace conv
}  // namespace dd
