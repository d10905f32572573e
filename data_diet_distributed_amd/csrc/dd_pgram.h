// Shifted-Gram ghost norms for small feature maps (dd_pgram.hip), called by the
// dd_conv_pegrad_sqnorm dispatcher (dd_pegrad.hip).
#pragma once
#include "dd_common.h"

namespace dd {

// geometry the kernel covers: 3x3 / pad 1 or 1x1 / pad 0, stride 1 or 2, <= 64 input and
// output positions (multiples of 4)
bool pgram_ok(const dd_conv_geom* g);

// sq[b] += ||grad_W||^2 of every example b < g->batch (no workspace)
int pgram_launch(const float* act, const float* gout, const dd_conv_geom* g,
                 const float* col_scale, float* sq, hipStream_t st);

// the quarter-tiled form for 3x3 / pad 1 / stride 1 on 16 x 16 maps (T = 256)
bool pgram_q_ok(const dd_conv_geom* g);
bool pgram_q_auto();

// partial[4 b + j] = the quarter-j sum of example b (reduced afterwards in a fixed order)
int pgram_q_launch(const float* act, const float* gout, const dd_conv_geom* g,
                   const float* col_scale, float* partial, hipStream_t st);

}  // namespace dd
