// Per-example weight-gradient norm of the network's input conv (dd_stem.hip), called by the
// dd_conv_pegrad_sqnorm dispatcher (dd_pegrad.hip).
#pragma once
#include "dd_common.h"

namespace dd {

// geometry the kernel covers: 3x3 / stride 1 / pad 1, cin * 9 <= 32, cout <= 64, width 8, 16
// or 32, H * W a multiple of 64
bool stem_ok(const dd_conv_geom* g);

// sq[b] += ||grad_W||^2 of every example b < g->batch (no workspace)
int stem_launch(const float* act, const float* gout, const dd_conv_geom* g,
                const float* col_scale, float* sq, hipStream_t st);

}  // namespace dd
