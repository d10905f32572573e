// conv3x3_r2_kernel padded-width instantiations (PW, see dd_conv_kern.h): the EL2N statistics
// launches of 3x3 stride-1 convs at widths that are not a tile width -- the ImageNet-stem
// network's 28x28 / 14x14 / 7x7 maps (reference models/resnet.py:35-63, Bottleneck conv2),
// which otherwise gather each tap's window per K chunk in the implicit GEMM (dd_conv1x1.hip).
#include "dd_conv_kern.h"

namespace dd {
namespace conv {

int dispatch_pw(int w, int pw, const Args& a, hipStream_t st) {
  if (w == 32 && pw == 1) return launch_r2_pw<32, 4, 1, 1>(a, st);
  if (w == 16 && pw == 2) return launch_r2_pw<16, 8, 1, 2>(a, st);
  if (w == 8 && pw == 2) return launch_r2_pw<8, 8, 2, 2>(a, st);
  if (w == 64 && pw == 1) return launch_narrow_pw<64, 2, 1, 1>(a, st);
  set_error("dd_conv3x3_forward: no padded-width tile of width %d (mode %d)", w, pw);
  return DD_EINVAL;
}

}  // namespace conv
}  // namespace dd
