/*
 * dd_capi.h — C-ABI of libdd.so, the MI355X (gfx950) Data Diet scoring/pruning kernels.
 *
 * Boundary: the reference has no FFI; its scoring path is the Python function
 *   sparse_loader(train_loader, train_samples, net, device, sparsity, batch_size, num_workers)
 *   (reference get_scores_and_prune.py:8-34).
 * Each entry point below replaces one step of that function (or one step the north star adds
 * to it); the file:line it replaces is cited on each declaration.  The Python host side
 * (data_diet_distributed_amd/get_scores_and_prune.py) keeps the reference signature and calls
 * these through ctypes (binding: INTEGRATION.md).
 *
 * Conventions (all entry points):
 *   - every pointer is a DEVICE pointer owned by the caller (torch tensors on the host side);
 *     no entry point allocates device memory: scratch comes from a caller workspace whose size
 *     is returned by the matching *_workspace_bytes query;
 *   - `stream` is a hipStream_t passed as void*; work is enqueued on it, nothing synchronises
 *     (entry points are graph-capturable);
 *   - return 0 on success, a negative DD_E* code on error; dd_last_error() returns a
 *     thread-local message for the last failing call on this thread;
 *   - stateless and reentrant; one process per GPU.
 */
#ifndef DD_CAPI_H
#define DD_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DD_OK 0
#define DD_EINVAL (-1)   /* bad argument (null pointer, negative size, unsupported shape) */
#define DD_ELAUNCH (-2)  /* HIP launch / runtime error */
#define DD_EWORKSPACE (-3) /* workspace too small */

/* ABI version, bumped on any signature change. */
int dd_abi_version(void);

/* Operand halves of the split MFMA convolutions (pack and forward must agree):
 *   DD_OPERANDS_BF16X3: v = hi + lo in bf16, products hi*hi + hi*lo + lo*hi with fp32
 *     accumulation (~2^-17 relative per product); any fp32 range.  The GraNd passes.
 *   DD_OPERANDS_F16X3: the same in fp16 (~2^-22 relative per product, at the same MFMA
 *     rate); operands must stay below 65504 in magnitude (values below 6.1e-5 carry an
 *     absolute error of at most 2^-25).  The EL2N forward (batch-normalised activations, raw
 *     weights): its ResNet-50 scores stay within the north star's 1e-3 of fp32.
 *     fp16 packs / launches exist for the statistics epilogue (every staging mode) and the
 *     generic run-time epilogue.
 * Weight scale: a pack holds W * scale and its forward multiplies the accumulators by
 * acc_scale = 1 / scale, both powers of two, so the product is exact.  bf16: scale 1.  fp16:
 * the host picks scale = 2^(13 - ceil(log2 max|W|)) so the weights' lo halves stay clear of
 * fp16's subnormal range (a small weight's lo half would otherwise carry ~2^-25 absolute
 * error: the ResNet GraNd forward's worst rows, tools/emulate_split_grand.py). */
#define DD_OPERANDS_BF16X3 0
#define DD_OPERANDS_F16X3 1

/* Message for the last non-zero return on the calling thread ("" if none). */
const char* dd_last_error(void);

/* ---------------------------------------------------------------------------------------- *
 * Input feed (reference data/loader.py:8-11 transform, applied per image in
 * MyDataset.__getitem__ :19-23 by the DataLoader workers of get_scores_and_prune.py:11):
 *   out[i, c, p] = (img[i, c, p] / 255 - mean[c]) / std[c]      (ToTensor + Normalize)
 * img: uint8 [n, C, HW] (CHW per image); out: fp32 [n, C, HW].  mean/std: host values.
 * ---------------------------------------------------------------------------------------- */
int dd_normalize_u8(const uint8_t* img, int64_t n, int32_t channels, int64_t hw,
                    const float* mean_host, const float* std_host, float* out, void* stream);

/* Same, gathering images by index: out[j] = normalize(img[index[j]]), j < n. */
int dd_normalize_u8_gather(const uint8_t* img, const int64_t* index, int64_t n,
                           int32_t channels, int64_t hw, const float* mean_host,
                           const float* std_host, float* out, void* stream);

/* Synthetic training set generated in HBM (replaces the dataset source of reference
 * data/loader.py:27-33 — torchvision CIFAR10(download=True) — for offline and ImageNet-shape
 * runs, BASELINE config 5).  Writes examples idx0 .. idx0+n-1 of the set named by `seed`:
 * img uint8 [n, C, h, w] and labels int64 [n] (labels may be NULL).  Every byte is a pure
 * function of (seed, global index, c, y, x), so shards generated on different ranks agree
 * with one whole-set generation; the hash is defined in dd_synth.hip and restated by
 * oracle/synth.py. */
int dd_synth_images_u8(uint64_t seed, int64_t idx0, int64_t n, int32_t channels, int32_t h,
                       int32_t w, int32_t num_classes, uint8_t* img, int64_t* labels,
                       void* stream);

/* ---------------------------------------------------------------------------------------- *
 * EL2N (reference get_scores_and_prune.py:16-18):
 *   p = softmax(logits[b, :]); e = p - onehot(label[b]); score[b] = ||e||_2
 * logits fp32 [B, C] row-major, labels int64 [B] in [0, C).
 * Outputs (each may be NULL):
 *   score[B]   : the EL2N score of each row (replaces the per-example .item() loop :19-20)
 *   e[B, C]    : the residual rows = d(sum CE)/d(logits), the GraNd backward seed; the
 *                label entry is written as -sum_{j != y} p_j (no p_y - 1 cancellation)
 *   accum[B]   : accum[b] += score[b]  (K-checkpoint ensemble running sum)
 *   bad_labels int32 [1] (device): += the number of rows whose label lies outside [0, C).
 * A label outside [0, C) is where the reference's one_hot(target, num_classes) raises (:17,
 * RuntimeError).  The kernel cannot raise, so such a row's score, accum term and e row are
 * NaN and the row is counted in bad_labels (one integer atomic add per bad row); the caller
 * reads the count back and raises (the engine does so once per job, after the score
 * all-gather, so every rank raises together).  ABI 9.
 * ---------------------------------------------------------------------------------------- */
int dd_el2n(const float* logits, const int64_t* labels, int64_t B, int32_t C,
            float* score, float* e, float* accum, int32_t* bad_labels, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * GraNd per-example gradient norms (north star (b); absent from the reference, which scores
 * with EL2N only — get_scores_and_prune.py:15-18; layers hooked: models/resnet.py:12-18,
 * 22-23, 40-47, 52-53, 71, 78).
 *
 * For a Conv2d with weight [Cout, Cin, kh, kw] (no bias, groups = 1), input activation
 * act fp32 NCHW [B, Cin, H, W] and output gradient gout fp32 NCHW [B, Cout, Ho, Wo]:
 *   sq_accum[b] += sum_{o, m} ( col_scale[o] * sum_t U_b[t, m] * gout[b, o, t] )^2
 * where U_b is the im2col of act[b] (t = output position, m = (c, ky, kx)).  col_scale may be
 * NULL (= 1); it carries a folded BatchNorm's gamma / sqrt(var + eps) when the forward ran
 * with BN folded into the conv.
 *   method DD_PEGRAD_DIRECT: per example G_b = U_b^T gout_b on MFMA, squared and summed in
 *     registers (2 T d_a d_g flop);
 *   method DD_PEGRAD_GHOST : sum_{t,t'} (U U^T)_{tt'} (gout gout^T)_{tt'} — the ghost-norm
 *     identity, both T x T Grams on MFMA (2 T^2 (d_a + d_g) flop);
 *   method DD_PEGRAD_AUTO  : the cheaper of the two for this geometry.
 * The result is deterministic (no float atomics): partial sums go to the workspace and are
 * reduced in a fixed order.
 * ---------------------------------------------------------------------------------------- */
#define DD_PEGRAD_AUTO 0
#define DD_PEGRAD_DIRECT 1
#define DD_PEGRAD_GHOST 2
#define DD_PEGRAD_DIRECT3X3 3 /* reported by dd_conv_pegrad_method only: the all-taps kernel */
#define DD_PEGRAD_PGRAM 4     /* reported only: ghost by shifted input-position Grams, for maps of
                                 <= 64 positions at DD_PREC_BF16X3: K_a = sum_tap P[p(t,tap)][p(t',tap)]
                                 with P = a^T a, so 2 (Ti^2 cin + To^2 cout) flop per example */
#define DD_PEGRAD_STEM 5      /* reported only: direct over the <= 32 im2col rows of an input conv
                                 with cin * 9 <= 32 (the network's first conv, 3 channels) at
                                 DD_PREC_BF16X3; bound by reading gout once */
#define DD_PEGRAD_DIRECT1X1 6 /* reported only: direct for a 1x1 conv (pad 0, stride 1 or 2) at
                                 DD_PREC_BF16X3: G = U^T g as a split-bf16 GEMM over positions */
#define DD_PEGRAD_PGRAM_Q 7   /* reported only: the shifted-Gram ghost for a 3x3 / pad 1 /
                                 stride 1 conv on a 16 x 16 map (T = 256, ResNet-18 layer2) at
                                 DD_PREC_BF16X3, tiled by quarters of the output positions (P
                                 does not fit LDS whole): 2 (Ti^2 cin + To^2 cout) flop per
                                 example; chosen by GHOST (AUTO keeps DIRECT3X3, measured faster
                                 on this shape: DESIGN.md §4.2) */

/* precision of the norm kernels:
 *   DD_PREC_FP32   exact fp32 MFMA (v_mfma_f32_32x32x2_f32 / 16x16x4_f32) everywhere;
 *   DD_PREC_BF16X3 split-bf16 MFMA where a kernel exists (3x3 stride-1 direct): each operand
 *                  v = hi + lo in bf16, products hi*hi + hi*lo + lo*hi accumulated in fp32
 *                  (~1e-5 relative per product; the GraNd tolerance is 1e-3). */
#define DD_PREC_FP32 0
#define DD_PREC_BF16X3 1

typedef struct dd_conv_geom {
  int64_t batch;   /* B */
  int32_t cin, h, w;      /* input  [B, cin, h, w] */
  int32_t cout, ho, wo;   /* output [B, cout, ho, wo] */
  int32_t kh, kw;         /* kernel */
  int32_t stride, pad;    /* symmetric stride / zero padding */
} dd_conv_geom;

/* Which kernel a (method, precision) request resolves to for this geometry:
 * DD_PEGRAD_DIRECT, DD_PEGRAD_GHOST, DD_PEGRAD_DIRECT3X3, DD_PEGRAD_PGRAM, DD_PEGRAD_STEM or
 * DD_PEGRAD_DIRECT1X1;
 * <0 on a bad argument. */
int dd_conv_pegrad_method(const dd_conv_geom* geom, int method, int precision);

size_t dd_conv_pegrad_workspace_bytes(const dd_conv_geom* geom, int method, int precision);

int dd_conv_pegrad_sqnorm(const float* act, const float* gout, const dd_conv_geom* geom,
                          const float* col_scale, int method, int precision, float* sq_accum,
                          void* workspace, size_t workspace_bytes, void* stream);

/* CIFAR head of the GraNd pass (reference models/resnet.py:94-96, avg_pool2d(out, 4) ->
 * linear), fp32 NCHW:
 *   dd_head_pool:     feat[b][c] = mean_p a[b][c][p]                          (a [B][C][hw])
 *   dd_head_backward: d[b][c][p] = scale * (sum_j e[b][j] W[j][c]) * (a[b][c][p] > 0)
 *     with e [B][ncls] the EL2N residual (the CE logit gradient), W [ncls][C] the classifier
 *     weight and scale = 1 / hw: the gradient w.r.t. the last block's pre-ReLU output, one
 *     pass over a (replaces e @ W, the broadcast divide and the ReLU mask as three torch ops). */
int dd_head_pool(const float* a, int64_t B, int32_t C, int32_t hw, float* feat, void* stream);
int dd_head_backward(const float* a, const float* e, const float* w, int64_t B, int32_t C,
                     int32_t hw, int32_t ncls, float scale, float* d, void* stream);

/* Classifier forward (reference models/resnet.py:96 `self.linear(out)`, nn.Linear :78):
 *   out[b][c] = sum_k feat[b][k] W[c][k] + (bias ? bias[c] : 0)
 * feat fp32 [B, d_in] (d_in <= 4096), W fp32 [d_out, d_in], bias fp32 [d_out] or NULL, out fp32
 * [B, d_out].  Each row is reduced in a fixed order from that row alone, so logits are
 * bitwise independent of B (chunk size, shard size, world size). */
int dd_linear_forward(const float* feat, const float* w, const float* bias, int64_t B,
                      int32_t d_in, int32_t d_out, float* out, void* stream);

/* Linear layer y = a W^T + bias (reference models/resnet.py:78, 96):
 *   sq_accum[b] += ||a_b||^2 * ||g_b||^2 + (has_bias ? ||g_b||^2 : 0)
 * act fp32 [B, d_in], gout fp32 [B, d_out] (for the classifier, gout = the EL2N residual e). */
int dd_linear_pegrad_sqnorm(const float* act, const float* gout, int64_t B, int32_t d_in,
                            int32_t d_out, int32_t has_bias, float* sq_accum, void* stream);

/* Eval-mode BatchNorm affine parameters (grand_params: all — the per-example gradient over
 * every parameter, as torch.func per-sample gradients define it; the BN layers are reference
 * models/resnet.py:13, 16, 24, 44, 46, 48, 53, 72).  With the BN output
 * out = gamma_c * xhat + beta_c and g = d loss / d out:
 *   sq_accum[b] += sum_c ( (sum_t g[b,c,t] * (v[b,c,t] - r[b,c,t] - beta_c)) / gamma_c )^2
 *                        + ( sum_t g[b,c,t] )^2
 * v fp32 [B, C, hw] must equal out + r wherever g != 0: the post-ReLU activation for a BN
 * followed by a ReLU (g vanishes where it clipped), or the block output with r = the
 * shortcut value for the last BN of a residual block (r may be NULL).  gamma_c != 0.
 * Deterministic (one fixed-order reduction per example). */
int dd_bn_pegrad_sqnorm(const float* v, const float* r, const float* g, int64_t B, int32_t C,
                        int64_t hw, const float* gamma, const float* beta, float* sq_accum,
                        void* stream);

/* ---------------------------------------------------------------------------------------- *
 * Backbone 3x3 / stride-1 / pad-1 convolution on split-bf16 MFMA (the ResNet convs of
 * reference models/resnet.py:12-15 (BasicBlock conv1 at stride 1, conv2) and :42-43
 * (Bottleneck conv2 at stride 1), i.e. 88% of ResNet-18 flops).  The reference runs them
 * through PyTorch (get_scores_and_prune.py:15); here they back the scoring passes.
 *   dd_conv3x3_pack: fp32 weights [cout][cin][3][3] -> bf16 hi/lo pack (device, caller-owned,
 *     dd_conv3x3_pack_bytes(out_ch, in_ch) bytes).  transpose_flip = 0 packs the forward conv
 *     (out_ch = cout, in_ch = cin); = 1 packs its backward-data conv (out_ch = cin,
 *     in_ch = cout, weights transposed and spatially flipped).  A forward pack with
 *     cin <= 5 (the input conv, reference models/resnet.py:71) uses the stem layout: the
 *     three kx taps of each channel become 3 cin pseudo-channels of the centre column, so
 *     the conv runs one K step per tap row; only dd_conv3x3_forward reads it.
 *   dd_conv3x3_forward: y[B][cout][h][w] = epi(conv(xf(x[B][cin][h][w]), packed)),
 *     xf(v)  = max(v * in_scale[g][c] + in_shift[g][c], in_relu ? 0 : -inf)   (input
 *              transform: the producer's train-mode BN + ReLU, reference models/resnet.py:28;
 *              identity when in_scale = in_shift = NULL), g = b / group_size;
 *     epi(v) = ((v + bias[o]) + residual) -> max(.,0) if relu -> 0 where !(mask_src > 0);
 *     bias / residual / mask_src may be NULL.  w in {8, 16, 32}; h a multiple of the
 *     row block (4 rows at w=32, 8 rows at w=16 and w=8), or 4x4.  fp32 accumulation;
 *     ~1e-5 relative vs fp32.
 *     stats (may be NULL): BN partial statistics of y over rows b < n_stat, laid out
 *     [G][cout][tiles_per_group][2] (sum, sum of squares) with G = ceil(B / group_size) and
 *     one partial per 32 consecutive positions of a group's examples (two images at 4x4):
 *     tiles_per_group = dd_conv3x3_tiles_per_group(h, w, group_size) = group_size*h*w/32;
 *     consumed by dd_bn_finalize with images_per_tile = max(1, 32 / (h*w)).  group_size
 *     must be even at 8x8 and a multiple of 4 at 4x4 when in_scale or stats is given.
 *     Padded-width launches (ABI 10): with the statistics epilogue alone (stats given; no
 *     bias, residual, masks or relu; cin > 5) the widths that are not a tile width also run
 *     here -- 32 < w <= 64 with w % 4 == 0 (any cout), and with cout padded to a multiple of
 *     128: 16 < w <= 32 with w % 4 == 0, 8 < w <= 16, and 4 < w <= 8 with h <= 8 and an even
 *     group_size; any h (the last row block may overhang): the ImageNet-stem network's
 *     56x56 / 28x28 / 14x14 / 7x7 maps (reference models/resnet.py:42-43).  The image is
 *     staged into the next tile width with zero columns / rows, which are never stored or
 *     counted; the partials keep the layout above on the padded grid: tiles_per_group =
 *     group_size * ceil(h / rb) * rb * wt / 32 ((rb, wt) = (2, 64), (4, 32), (8, 16),
 *     (8, 8)), images_per_tile 1.  DD_CONV_PW=0 turns them off.
 *   dd_conv3x3_tiles_per_group: partials per BN group of the stats layout (< 0 if
 *     unsupported).
 *   dd_conv3x3_padded_supported: 1 where a statistics launch of this shape takes the
 *     padded-width tiles (not a native shape; see above), else 0.
 *   mask_out / mask_in (may be NULL; dd_conv3x3_mask_bytes(B, cout, h, w) bytes): the ReLU
 *     mask (y > 0) in the kernel's fragment order, 1 bit per output.  A launch writing
 *     mask_out and a later launch of the same geometry (B, h, w, output channels) reading
 *     mask_in (in place of mask_src) see the same (example, channel, position) at the same
 *     bit, so the GraNd backward reads 1/32 of the bytes of the fp32 activation it masks by
 *     (reference BasicBlock ReLUs, models/resnet.py:28, 31).
 * ---------------------------------------------------------------------------------------- */
size_t dd_conv3x3_pack_bytes(int32_t out_channels, int32_t in_channels);
int dd_conv3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t transpose_flip,
                    int32_t operands, float scale, void* packed, void* stream);
int dd_conv3x3_tiles_per_group(int32_t h, int32_t w, int32_t group_size);
int dd_conv3x3_padded_supported(int32_t h, int32_t w, int32_t cin, int32_t cout,
                                int32_t group_size);
size_t dd_conv3x3_mask_bytes(int64_t B, int32_t cout, int32_t h, int32_t w);
int dd_conv3x3_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                       const void* packed, int32_t cout, const float* bias,
                       const float* residual, const float* mask_src, int32_t relu,
                       const float* in_scale, const float* in_shift, int32_t in_relu,
                       int32_t group_size, int64_t n_stat, float* stats, uint16_t* mask_out,
                       const uint16_t* mask_in, float* y, int32_t operands, float acc_scale,
                       void* stream);
/* Residual-unit output fused into the next unit's first conv (EL2N pass, train-mode BN):
 *   dd_conv3x3_forward_unit_input: x = max(y_prev * in_scale[g][c] + in_shift[g][c] + R, 0)
 *     with R = 0 (res NULL: the stem's BN + ReLU), res (identity shortcut) or res *
 *     res_scale[g][c] + res_shift[g][c] (the projection shortcut's BN), i.e. reference
 *     models/resnet.py:31-32 (out = bn2(conv2(.)); out += shortcut(x); relu(out)) and :89
 *     (relu(bn1(conv1(x)))), computed while the conv stages it: x is written to x_out
 *     [B][cin][h][w] once (the unit's output, which the next unit adds as its shortcut) and
 *     y = conv(x) with BN statistics as dd_conv3x3_forward (stats required, group_size as
 *     there).  Replaces a dd_bn_apply pass over y_prev and res plus the conv's read of its
 *     output.  x_out is bitwise dd_bn_apply's output, y bitwise dd_conv3x3_forward's on it.
 *   dd_conv3x3_unit_input_supported: 1 where the fused form exists (the scoring tiles: 32x32,
 *     and 16x16 / 8x8 with cout a multiple of 128; cin > 5), else 0. */
int dd_conv3x3_unit_input_supported(int32_t h, int32_t w, int32_t cin, int32_t cout,
                                    int32_t group_size);
int dd_conv3x3_forward_unit_input(const float* y_prev, const float* in_scale,
                                  const float* in_shift, const float* res,
                                  const float* res_scale, const float* res_shift, float* x_out,
                                  int64_t B, int32_t cin, int32_t h, int32_t w,
                                  const void* packed, int32_t cout, int32_t group_size,
                                  int64_t n_stat, float* stats, float* y, int32_t operands,
                                  float acc_scale, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * The ImageNet stem's 7x7 / stride 2 / pad 3 conv, 3 -> cout <= 64 channels (reference
 * models/resnet.py ImageNet stem; BASELINE config 5), the EL2N launch shape (ABI 10):
 *   y [B][cout][h/2][w/2] = conv(x [B][3][h][w]) with BN partial statistics over rows b < n_stat
 *   in groups of group_size, one partial per (group, channel, 32-position fragment of an
 *   output-row pair): tiles_per_group = dd_stem7_tiles_per_group(h, w, group_size) =
 *   group_size * ceil(h / 4) * 8, images_per_tile 1 for dd_bn_finalize.
 * h, w even, w / 2 a multiple of 4 and at most 128.  The staged rows replace the implicit
 * GEMM's per-chunk gathers (dd_conv_gemm_forward's dense mode).
 *   dd_stem7_pack: W [cout][3][7][7] -> hi/lo fragment pack (dd_stem7_pack_bytes() bytes) in
 *     the `operands` halves (scale: a power of two for fp16, 1 for bf16; the forward takes its
 *     inverse as acc_scale).
 * ---------------------------------------------------------------------------------------- */
size_t dd_stem7_pack_bytes(void);
int dd_stem7_pack(const float* w, int32_t cout, int32_t operands, float scale, void* packed,
                  void* stream);
int dd_stem7_supported(int32_t h, int32_t w, int32_t cin, int32_t cout, int32_t group_size);
int dd_stem7_tiles_per_group(int32_t h, int32_t w, int32_t group_size);
int dd_stem7_forward(const float* x, int64_t B, int32_t h, int32_t w, const void* packed,
                     int32_t cout, int32_t group_size, int64_t n_stat, float* stats, float* y,
                     int32_t operands, float acc_scale, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * ResNet downsampling head (reference models/resnet.py:12 BasicBlock conv1 at stride 2 and
 * :20-23 its 1x1 stride-2 projection shortcut), split-bf16 MFMA, one launch for both:
 *   y    = epi(conv3x3_s2_p1(x, packed3x3))   [B][cout][ho][wo], x [B][cin][2 ho][2 wo]
 *   y_sc = epi_sc(conv1x1_s2(x, packed1x1))   (packed1x1 / y_sc NULL: no shortcut)
 * epi(v) = relu?(v + bias[o]) (bias may be NULL); stats / stats_sc: grouped BN partials as
 * for dd_conv3x3_forward with tiles_per_group = dd_down_tiles_per_group(ho, wo, group_size).
 * The shortcut reads exactly the centre tap of the stride-2 window, so it shares the staged
 * input and B fragments.  Output shapes: wo = 32 with even ho, wo = 16 with ho % 4 == 0,
 * 8x8, 4x4.  Padded-width heads (ABI 10): the statistics launch of a stride-2 conv alone (no
 * shortcut, bias or relu; cin > 64; cout padded to a multiple of 128), the ResNet-50
 * Bottleneck conv2 at stride 2 (reference models/resnet.py:42-43), also runs at 16 < wo <= 32
 * with wo % 4 == 0, 8 < wo <= 16 with wo even, and 4 < wo <= 8, any ho: the ImageNet-stem
 * network's 56 -> 28, 28 -> 14, 14 -> 7 heads.  The map is staged into the next tile width
 * with zero columns / rows, never stored or counted; tiles_per_group = group_size *
 * ceil(ho / rb) * 2 (rb = 2 / 4 / 8), images_per_tile 1.  DD_DOWN_PW=0 turns them off.
 *   dd_down_padded_supported: 1 where such a launch takes the padded-width head, else 0.
 *   dd_conv1x1_pack: 1x1 weights [cout][cin] -> hi/lo fragment pack in the `operands` halves
 *     (dd_conv1x1_pack_bytes(out_ch, in_ch)); transpose = 1 packs W^T (out = cin, in = cout).
 * `operands` (DD_OPERANDS_*) of the forward entry points must be the packs'; the fp16 form
 * exists for the statistics epilogue (with or without the staging transform) and the run-time
 * epilogue.
 * ---------------------------------------------------------------------------------------- */
size_t dd_conv1x1_pack_bytes(int32_t out_channels, int32_t in_channels);
int dd_conv1x1_pack(const float* w, int32_t cout, int32_t cin, int32_t transpose,
                    int32_t operands, float scale, void* packed, void* stream);
int dd_down_tiles_per_group(int32_t ho, int32_t wo, int32_t group_size);
int dd_down_padded_supported(int32_t ho, int32_t wo, int32_t cin, int32_t cout,
                             int32_t group_size);
int dd_down_forward(const float* x, int64_t B, int32_t cin, int32_t ho, int32_t wo,
                    const void* packed3x3, const void* packed1x1, int32_t cout,
                    const float* bias, int32_t relu, float* stats, float* y,
                    const float* bias_sc, int32_t relu_sc, float* stats_sc, float* y_sc,
                    int32_t group_size, int64_t n_stat, int32_t operands, float acc_scale,
                    float acc_scale_sc, void* stream);
/* The downsampling head with its input computed while staging (EL2N pass, train-mode BN;
 * replaces a dd_bn_apply pass and the head's read of its output):
 *   dd_down_forward_unit_input: x = max(y_prev * in_scale[g][c] + in_shift[g][c] (+ res), 0),
 *     then y / y_sc and their BN statistics as dd_down_forward (stats required; no bias or
 *     ReLU epilogue).  With res (the previous BasicBlock unit's identity shortcut) x is that
 *     unit's output relu(bn2(conv2(.)) + shortcut) (reference models/resnet.py:31-32), which
 *     only this head reads, so it is never written; res needs packed1x1 / y_sc / stats_sc (the
 *     stage head's projection).  Without res and without a shortcut, x is the producer's
 *     BN + ReLU (a Bottleneck's stride-2 conv2, reference :42).  x is bitwise dd_bn_apply's
 *     output, y / y_sc / stats bitwise dd_down_forward's on it. */
int dd_down_forward_unit_input(const float* y_prev, const float* in_scale,
                               const float* in_shift, const float* res, int64_t B, int32_t cin,
                               int32_t ho, int32_t wo, const void* packed3x3,
                               const void* packed1x1, int32_t cout, float* stats, float* y,
                               float* stats_sc, float* y_sc, int32_t group_size,
                               int64_t n_stat, int32_t operands, float acc_scale,
                               float acc_scale_sc, void* stream);
/* Backward-data of the head (the GraNd backward through models/resnet.py:12, :20-23):
 *   dx = (conv3x3_s2^T(dh, W) + conv1x1_s2^T(dz, Ws)) * (mask_src > 0)   [B][cin][2ho][2wo]
 * dh, dz [B][cout][ho][wo] (dz / packed1x1_t NULL: no shortcut; mask_src NULL: no mask);
 * packed3x3_t = dd_conv3x3_pack(W, transpose_flip = 1), packed1x1_t = dd_conv1x1_pack(Ws,
 * transpose = 1).  Computed as the 4 sub-pixel parity classes of dx (no zero insertion). */
int dd_down_backward(const float* dh, const float* dz, int64_t B, int32_t cout, int32_t ho,
                     int32_t wo, const void* packed3x3_t, const void* packed1x1_t, int32_t cin,
                     const float* mask_src, const uint32_t* mask_bits, float* dx,
                     void* stream);

/* The ReLU-backward mask of a downsampling head's input as bits (the GraNd backward, reference
 * models/resnet.py:31 relu of the previous block's output): dd_down_backward takes either the
 * fp32 tensor (mask_src: dx = 0 where !(mask_src > 0)) or mask_bits = plane bits, bit p & 31
 * of word ((b * cin + c) * 4 ho wo + p) >> 5 (wo in {4, 8, 16}), one 32nd of its bytes.
 *   dd_conv3x3_mask_plane_bits: the mask_out words of a dd_conv3x3_forward launch (B, cout,
 *     h, w, ungrouped) -> plane bits [B * cout * h * w / 32] (h * w a multiple of 32). */
int dd_conv3x3_mask_plane_bits(const uint16_t* mask, int64_t B, int32_t cout, int32_t h,
                               int32_t w, uint32_t* bits, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * 1x1 convolution on split-bf16 MFMA (ResNet-50 Bottleneck conv1 / conv3, reference
 * models/resnet.py:40, 44, and the 1x1 projection shortcuts :49-54 at stride 1 or 2), the
 * GEMM y[b][o][p] = sum_c W[o][c] xf(x[b][c][stride * p]) over the flattened (b, p) space:
 *   packed = dd_conv1x1_pack(W, transpose = 0) (forward) or (W, transpose = 1) (backward-data:
 *     out = cin, in = cout, stride 1);
 *   epi(v) = ((v + bias[o]) + residual + up2(res_up2)) -> max(.,0) if relu -> 0 where
 *     !(mask_src > 0); up2(r)[b][o][y][x] = r[b][o][y/2][x/2] at even (y, x), else 0 (the
 *     backward of a stride-2 projection fused into the block-input gradient);
 *   xf / in_scale / in_shift / in_relu / group_size / n_stat / stats exactly as
 *     dd_conv3x3_forward, with tiles_per_group = dd_conv1x1_tiles_per_group(ho, wo,
 *     group_size) = group_size * ho * wo / 64 (requires group_size * ho * wo % 128 == 0):
 *     one partial per 64 consecutive positions of the group's flattened (example, position)
 *     space, consumed by dd_bn_finalize with images_per_tile = -64.
 * Any h, w (even at stride 2); output [B][cout][h / stride][w / stride].
 * ---------------------------------------------------------------------------------------- */
int dd_conv1x1_tiles_per_group(int32_t ho, int32_t wo, int32_t group_size);
int dd_conv1x1_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                       int32_t stride, const void* packed, int32_t cout, const float* bias,
                       const float* residual, const float* res_up2, const float* mask_src,
                       int32_t relu, const float* in_scale, const float* in_shift,
                       int32_t in_relu, int32_t group_size, int64_t n_stat, float* stats,
                       float* y, int32_t operands, float acc_scale, void* stream);
/* A ResNet-50 unit's output fused into the next unit's first (1x1, stride-1) conv (ABI 8;
 * the EL2N forward of configs 4-5, reference models/resnet.py:57-63): the conv's input is
 *   xout = relu(y_prev * scale + shift [+ xres (* xres_scale + xres_shift)])
 * computed while staging in dd_bn_apply's arithmetic order (bitwise that pass), written to xout
 * once (the next unit's residual / projection input), and y / stats are those of
 * dd_conv1x1_forward(xout, ...) with the grouped BN statistics epilogue (no bias, residual,
 * mask or ReLU on y). scale / shift / xres_* are [G][cin] per group_size rows; xres NULL: no
 * residual; xres_scale / xres_shift NULL: an identity residual. Needs h * w % 4 == 0 and
 * 16-byte aligned tensors (DD_EINVAL otherwise). */
int dd_conv1x1_forward_unit_input(const float* y_prev, const float* scale, const float* shift,
                                  const float* xres, const float* xres_scale,
                                  const float* xres_shift, float* xout, int64_t B, int32_t cin,
                                  int32_t h, int32_t w, const void* packed, int32_t cout,
                                  int32_t group_size, int64_t n_stat, float* stats, float* y,
                                  int32_t operands, float acc_scale, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * Any kh x kw convolution (stride 1 or 2, zero padding `pad`) as an implicit GEMM on the same
 * kernel: the ResNet-50 ImageNet-stem network of config 5 (reference models/resnet.py: the
 * 7x7/2 stem conv and the 3x3 convs at 56 / 28 / 14 / 7, stride 1 and 2), forward only.
 *   packed = dd_conv_gemm_pack(W [cout][cin][kh][kw]) (dd_conv_gemm_pack_bytes bytes): K is
 *     (tap, channel) tap-major with each tap's channels padded to 32, or (channel, tap) dense
 *     (PyTorch's weight order, padded to 32) when dd_conv_gemm_dense(cin, kh, kw) = 1
 *     (inputs with fewer than 32 channels: the 7x7 stem's K = 147 in 5 chunks, not 49);
 *   y[B][cout][ho][wo], ho = (h + 2 pad - kh) / stride + 1 (likewise wo),
 *     = epi(sum_{c,ky,kx} W[o][c][ky][kx] xf(x)[b][c][ho*s + ky - pad][wo*s + kx - pad]),
 *     xf applied before the zero padding (a dense pack takes no xf); bias / residual / relu /
 *     in_* / group_size / n_stat / stats exactly as dd_conv1x1_forward.
 * ---------------------------------------------------------------------------------------- */
int dd_conv_gemm_dense(int32_t cin, int32_t kh, int32_t kw);
size_t dd_conv_gemm_pack_bytes(int32_t out_channels, int32_t in_channels, int32_t kh,
                               int32_t kw);
int dd_conv_gemm_pack(const float* w, int32_t cout, int32_t cin, int32_t kh, int32_t kw,
                      int32_t operands, float scale, void* packed, void* stream);
int dd_conv_gemm_forward(const float* x, int64_t B, int32_t cin, int32_t h, int32_t w,
                         int32_t kh, int32_t kw, int32_t stride, int32_t pad,
                         const void* packed, int32_t cout, const float* bias,
                         const float* residual, int32_t relu, const float* in_scale,
                         const float* in_shift, int32_t in_relu, int32_t group_size,
                         int64_t n_stat, float* stats, float* y, int32_t operands,
                         float acc_scale, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * Grouped train-mode BatchNorm (the reference's scoring forward runs BN with batch
 * statistics: train.py:59-63 never calls .eval(); BN layers models/resnet.py:13-16, 72).
 * One launch carries G = ceil(B / group_size) pinned batches, each normalised with its own
 * statistics; rows b >= n_valid are excluded (a ragged final batch).
 *   dd_channel_stats: partials of any NCHW tensor y [B][C][hw] in the layout above with
 *     tiles_per_group = group_size, images_per_tile = 1, row_tiles = 1.
 *   dd_bn_finalize: per (group, channel): mean, biased variance over count(g) * hw values
 *     (count(g) = clamp(n_valid - g * group_size, 0, group_size); the first
 *     ceil(count / images_per_tile) * row_tiles tiles; images_per_tile = -T < 0: tiles of T
 *     consecutive positions of the group's flattened (example, position) space, the first
 *     ceil(count * hw / T) of them), summed in double in a fixed order;
 *     scale = gamma / sqrt(var + eps), shift = beta - mean * scale  ([G][C] fp32 each).
 *   dd_bn_apply: out = relu?(y * scale + shift + R) with R = 0 (residual NULL), the raw
 *     residual, or max?(residual * res_scale + res_shift) (its own BN, res_relu);
 *     reference BasicBlock tail models/resnet.py:30-31.  pool_out [B][C] (may be NULL):
 *     the spatial mean of out (the CIFAR head avg_pool2d(out, 4), :94); out may then be NULL.
 *     Pooling needs hw / 4 a power of two <= 64 and 16-B aligned tensors.
 * ---------------------------------------------------------------------------------------- */
int dd_channel_stats(const float* y, int64_t B, int32_t C, int64_t hw, int32_t group_size,
                     int64_t n_stat, float* stats, void* stream);
int dd_bn_finalize(const float* stats, int64_t n_groups, int32_t group_size, int64_t n_valid,
                   int32_t tiles_per_group, int32_t images_per_tile, int32_t row_tiles,
                   int32_t C, int64_t hw, const float* gamma, const float* beta, float eps,
                   float* scale, float* shift, void* stream);
/* dd_bn_apply_maxpool: the ImageNet stem tail, relu(y * scale + shift) then max_pool2d(3,
 *   stride 2, padding 1) in one pass: out [B][C][(h-1)/2+1][(w-1)/2+1] (the 112x112 stem
 *   output is never written at full resolution). */
int dd_bn_apply_maxpool(const float* y, int64_t B, int32_t C, int32_t h, int32_t w,
                        int32_t group_size, const float* scale, const float* shift,
                        float* out, void* stream);
int dd_bn_apply(const float* y, int64_t B, int32_t C, int64_t hw, int32_t group_size,
                const float* scale, const float* shift, const float* residual,
                const float* res_scale, const float* res_shift, int32_t res_relu, int32_t relu,
                float* out, float* pool_out, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * K-checkpoint ensemble (north star (c); the reference scores one hard-coded checkpoint,
 * train.py:61, train_sparse.py:23, ddp.py:72).
 *   dd_sqrt_accumulate : accum[b] += sqrt(sq[b])       (GraNd norm of one checkpoint)
 *   dd_ensemble_finalize: out[i] = accum[i] / K          (mean over K checkpoints)
 * ---------------------------------------------------------------------------------------- */
int dd_sqrt_accumulate(const float* sq, int64_t B, float* accum, void* stream);
int dd_ensemble_finalize(const float* accum, int64_t n, int32_t K, float* out, void* stream);

/* ---------------------------------------------------------------------------------------- *
 * Keep-set selection (reference get_scores_and_prune.py:22-24):
 *   samples = int((1 - sparsity) * train_samples)                          (:22)
 *   indices = [i for i, s in sorted(scores, key=s, reverse=True)[:samples]]  (:23-24)
 * dd_keep_count returns `samples` with the reference's IEEE-double truncation.
 *
 * dd_select_topk: keys fp32 [n] (key i belongs to index i), k in [0, n].  Writes
 *   idx_out int64 [k] : the k indices of largest key, ordered by key descending and, among
 *                       equal keys, by ascending index (Python's stable sort with
 *                       reverse=True keeps visit order; +0.0 == -0.0 as in Python);
 *   thr_out fp32 [1]  : the k-th largest key (NULL allowed; unspecified when k == 0).
 *   nan_count_out int32 [1] (device, NULL allowed): number of NaN keys.  The reference's
 *                       sort is undefined on NaN; here NaN ranks below every number.  The
 *                       host wrapper reads this after the call and raises (no sync inside).
 * One read of the keys for an 11-bit top-digit histogram (the threshold bin), a second that
 * compacts the m >= k keys in or above that bin in index order, then three stable LSD radix
 * passes over them on the low ceil(R / 3) bits of key - base (R = the survivors' key range
 * in bits, decided on the device); n < 2^31.  Workspace: dd_select_workspace_bytes(n), 16-byte
 * aligned (its per-call state is cleared on the stream: reusable across calls and graph replays).
 * ---------------------------------------------------------------------------------------- */
int64_t dd_keep_count(int64_t train_samples, double sparsity);

size_t dd_select_workspace_bytes(int64_t n);

int dd_select_topk(const float* keys, int64_t n, int64_t k, int64_t* idx_out, float* thr_out,
                   int32_t* nan_count_out, void* workspace, size_t workspace_bytes,
                   void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DD_CAPI_H */
