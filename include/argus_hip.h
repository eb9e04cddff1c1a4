/*
 * argus_hip.h — C ABI of libargus_hip.so, the MI355X (gfx950) kernels behind the argus training
 * hot path. Plain C: raw device pointers, sizes, an opaque HIP stream; no torch types.
 *
 * The reference (pculbertson/argus) has no FFI; its device work is dispatched implicitly through
 * torchvision / pypose / torch.optim / DDP. Each entry point below replaces one of
 * those implicit kernels and names the reference call site it stands in for. The Python host layer
 * (argus_amd/_lib.py, ctypes) binds exactly these symbols; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Activations are NHWC, channel-contiguous, dtype ARGUS_F32 or ARGUS_BF16.
 *  - Conv weights are OHWI ("KRSC"): w[k][r][s][c]. The stem (7x7, C=3) uses a padded compute layout
 *    w[k][r(8)][s(8)][c(4)] (r=7, s=7, c=3 zero) and an NHWC4 input (channel 3 zero).
 *  - Statistics, losses, gradients of parameters and optimizer state are fp32.
 *  - Every call enqueues on `stream` (hipStream_t; NULL = legacy default) and returns 0 on success or
 *    a nonzero code; argus_last_error() then describes it. The library never allocates device memory:
 *    callers pass workspaces sized by the *_bytes() queries. No call synchronises the device.
 */
#ifndef ARGUS_HIP_H
#define ARGUS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* argus_stream_t; /* hipStream_t */

/* ARGUS_FP8 (conv fwd / dgrad and weight-prep entry points): bf16 activations, GEMM operands in OCP
 * MX-fp8 (e4m3 + one E8M0 scale per 32 K-elements of a row) for the MFMA
 * v_mfma_scale_f32_16x16x128_f8f6f4 where the conv pass allows it (reduction channels % 128 == 0, not
 * the stem): the activation operand (and a BN-backward apply prologue) is quantized while staging, the
 * weights are the pre-quantized copies argus_conv_weight_prep(_batch) writes with ARGUS_FP8 (e4m3 rows
 * [rows][cols] then scales [rows][cols/32], in the bf16 copy's buffer). The other passes and every
 * non-conv entry point (pass ARGUS_BF16) run bf16. */
enum { ARGUS_F32 = 0, ARGUS_BF16 = 1, ARGUS_FP8 = 2 };
enum { ARGUS_OK = 0, ARGUS_ERR_ARG = 1, ARGUS_ERR_SHAPE = 2, ARGUS_ERR_HIP = 3 };

/* One override of the kernel-selection policy (keys: argus_conv_policy_default). */
typedef struct {
  int32_t key, value;
} argus_tuning;

typedef struct {
  int32_t n, h, w; /* images, input spatial */
  int32_t c;       /* input channels (3 for the stem) */
  int32_t k;       /* output channels */
  int32_t r, s;    /* filter size */
  int32_t stride, pad;
  int32_t ho, wo; /* output spatial */
  int32_t stem;   /* 1: the 7x7/2 stem (NHWC4 input, padded weights) */
  /* Optional per-call overrides of the library's kernel-selection policy (experiments, autotuning and
   * the kernel-coverage tests): n_tuning entries of `tuning`; 0 / NULL = the library defaults. The
   * library keeps no mutable selection state: a call sees its own overrides and nothing else. */
  int32_t n_tuning;
  const argus_tuning* tuning;
} argus_conv_desc;

int argus_abi_version(void);
const char* argus_last_error(void);

/* ---- input / weight layout ------------------------------------------------------------------ */
/* (B,3*ncam,H,W) fp32 NCHW -> (B*ncam,H,W,4) NHWC4 of dtype; replaces the reshape at
 * argus/models.py:81 plus the layout change cuDNN does internally. */
int argus_images_to_nhwc4(int dtype, int64_t nimg, int h, int w, const float* x, void* out,
                          argus_stream_t stream);
/* Same, from uint8 images (B,3*ncam,H,W) as CameraCubePoseDataset(uint8=True) yields them: the
 * `.to(torch.float32) / 255.0` of argus/data.py:214-215 runs on the device (4x less H2D traffic). */
int argus_images_u8_to_nhwc4(int dtype, int64_t nimg, int h, int w, const uint8_t* x, void* out,
                             argus_stream_t stream);
/* fp32 master weight -> compute copies: w_fwd[k][r][s][c] (dtype; padded [k][8][8][4] for the
 * stem) and w_dgrad[c][r][s][k] (dtype; ignored for the stem). The master is read with element
 * strides {sk, sc, sr, ss} (so an OIHW nn.Parameter or a channels-last view both work);
 * strides == NULL means OHWI contiguous. */
int argus_conv_weight_prep(const argus_conv_desc* d, int dtype, const float* w_master,
                           const int64_t* strides, void* w_fwd, void* w_dgrad,
                           argus_stream_t stream);

/* ---- convolution (torchvision Conv2d, bias=False; models.py:43) ------------------------------ */
/* Batched weight_prep (one launch for a whole network): the host writes a table of `count`
 * conversions (argus_conv_weight_prep_table: per conv its descriptor, fp32 master pointer and
 * element strides {sk, sc, sr, ss} (NULL strides = OHWI contiguous), w_fwd and w_dgrad destinations
 * (w_dgrad array NULL or entry ignored for the stem)) into host_table, copies it to device memory
 * once, and then argus_conv_weight_prep_batch does what argus_conv_weight_prep does for every entry.
 * The table holds raw device pointers: rebuild it if any of them changes. */
size_t argus_conv_weight_prep_table_bytes(int count);
int argus_conv_weight_prep_table(int count, const argus_conv_desc* descs, const float* const* w_master,
                                 const int64_t* strides, void* const* w_fwd, void* const* w_dgrad,
                                 void* host_table, size_t table_bytes, int* nblocks);
int argus_conv_weight_prep_batch(int dtype, int count, const void* device_table, int nblocks,
                                 argus_stream_t stream);
/* y = conv(x', w) where x' = relu(x*pro_scale+pro_shift) per input channel when pro_scale != NULL
 * (the producer's BatchNorm+ReLU applied while staging; zero padding stays zero), else x.
 * If stat_part != NULL, per-(row-tile, channel) {sum, M2} of y (fp32 accumulators, before
 * rounding; M2 about the tile mean) are written: float2[argus_conv_fwd_stat_rows(d)][k], each row
 * tile covering argus_conv_fwd_stat_tile(d) output pixels (the last one possibly fewer); a negative
 * stat tile (ragged tiling) also writes int32 pixel counts[rows] after them, so stat_part must then
 * hold 2*rows*k floats + rows ints. */
int argus_conv_fwd(const argus_conv_desc* d, int dtype, const void* x, const void* w_fwd, void* y,
                   const float* pro_scale, const float* pro_shift, float* stat_part,
                   argus_stream_t stream);
/* y == NULL (bf16, not the stem, stat_part given): statistics only, nothing stored (ABI 14; the
 * bottleneck's conv3 before argus_conv_fwd_bn_out). */
/* argus_conv_fwd with its BN+ReLU prologue (pro_scale / pro_shift required) that also stores the
 * staged input x' = relu(x*pro_scale+pro_shift) to x_out, bit-identical to argus_bn_apply(relu = 1)
 * of x (ABI 16; 1x1 stride-1 convs, bf16 or fp32): the bottleneck's conv3 statistics pass applies bn2
 * to y2 while staging it and writes a2 (the operand of the fused tail and of conv3's weight gradient),
 * replacing the separate bn2 apply pass of torchvision's Bottleneck.forward (argus/models.py:43). */
int argus_conv_fwd_apply_out(const argus_conv_desc* d, int dtype, const void* x, const void* w_fwd, void* y,
                             const float* pro_scale, const float* pro_shift, float* stat_part, void* x_out,
                             argus_stream_t stream);
/* Bottleneck tail in one forward pass (ABI 14; replaces conv3 + bn3 + the residual add + ReLU of
 * torchvision's Bottleneck.forward, argus/models.py:43 -> torchvision resnet.py, in train mode after
 * argus_bn_finalize of bn3, or eval mode with argus_bn_eval_coeffs): the 1x1 stride-1 conv's C tile t
 * (rounded to bf16, as argus_conv_fwd stores it) gives out = relu(t*scale + shift + res'), res' = res *
 * res_scale + res_shift when res_scale != NULL (the downsample BN) else res, with argus_bn_apply's
 * mask bits (one byte per 16-byte chunk). Bit-identical to argus_conv_fwd + argus_bn_apply. y: optional
 * store of t (NULL: not stored). bf16 only; every tensor NHWC. */
int argus_conv_fwd_bn_out(const argus_conv_desc* d, int dtype, const void* x, const void* w_fwd,
                          const float* scale, const float* shift, const void* res, const float* res_scale,
                          const float* res_shift, void* out, uint8_t* mask_bits, void* y, argus_stream_t stream);
int argus_conv_fwd_stat_rows(const argus_conv_desc* d, int dtype);
int argus_conv_fwd_stat_tile(const argus_conv_desc* d, int dtype);
/* The partial layout (rows, tile as above) of a statistics-only argus_conv_fwd (y == NULL, no
 * prologue; ABI 16): bf16 1x1 stride-1 convs with 64..512 input channels run on a persistent kernel
 * (policy key 44) that writes one {sum, M2} row per row split and the int32 pixel counts after them
 * (negative tile: ragged rows); other convs as argus_conv_fwd_stat_rows / _stat_tile. */
int argus_conv_fwd_stats_only_rows(const argus_conv_desc* d, int dtype);
int argus_conv_fwd_stats_only_tile(const argus_conv_desc* d, int dtype);
/* The BatchNorm train-mode finalize of a forward conv's statistics (argus_bn_finalize's arguments
 * past its partial layout), for argus_conv_fwd_fin. workspace: argus_bn_workspace_bytes(k), zeroed once
 * (every call leaves it zeroed); running_mean / running_var / num_batches_tracked may be NULL. */
typedef struct argus_bn_fwd_fin {
  void* workspace;
  const float* gamma;
  const float* beta;
  float eps;
  float momentum;
  float* running_mean;
  float* running_var;
  int64_t* num_batches_tracked;
  float* mean;
  float* invstd;
  float* scale;
  float* shift;
} argus_bn_fwd_fin;
/* argus_conv_fwd (stat_part required) followed by argus_bn_finalize of its partials (the layout
 * argus_conv_fwd_stat_rows / _tile, or _stats_only_rows / _tile when y == NULL), with the finalize
 * folded into the conv's last-arriving workgroups where the producing kernel's row tiles align with
 * argus_bn_finalize's merge groups (otherwise it is launched after the conv): mean, invstd, scale, shift
 * and the running statistics are bit-identical to the two calls either way (ABI 18). Replaces the
 * BatchNorm2d train forward's statistics pass of torchvision's Bottleneck (argus/models.py:43). */
int argus_conv_fwd_fin(const argus_conv_desc* d, int dtype, const void* x, const void* w_fwd, void* y,
                       const float* pro_scale, const float* pro_shift, float* stat_part,
                       const argus_bn_fwd_fin* fin, argus_stream_t stream);
/* Bytes a stat_part buffer needs for argus_conv_fwd of d (stats_only = 0) or for its statistics-only
 * form (y == NULL, stats_only = 1): 2*rows*k floats plus, for a ragged tiling (negative tile), int32
 * counts[rows] after them (ABI 17). Size every statistics workspace with it; rows*k*2 floats alone is
 * too small for the ragged stem and the persistent statistics-only forward. 0 for a bad descriptor. */
size_t argus_conv_fwd_stat_part_bytes(const argus_conv_desc* d, int dtype, int stats_only);
/* dx = dgrad(dy, w_dgrad) [+ addend]: when addend != NULL (same NHWC layout as dx; may be dx itself
 * for in-place accumulation) it is added, element-wise masked by addend_mask when that is non-NULL
 * (the bn_apply ReLU mask: the residual path of a bottleneck, dx += relu'(out) * dout). */
int argus_conv_dgrad(const argus_conv_desc* d, int dtype, const void* dy, const void* w_dgrad,
                     void* dx, const void* addend, const uint8_t* addend_mask, argus_stream_t stream);
/* dgrad whose output feeds the backward of a BatchNorm (+ReLU): the BN-backward reduction
 * (argus_bn_bwd_reduce) runs in the dgrad epilogue instead of as its own pass over dz.
 * With v = dgrad(dy, w_dgrad) [+ addend] (addend unmasked, may alias dm), the kernel stores
 * dm = v * mask (mask_mode 2: y*scale+shift > 0, the BN's own ReLU; 3: mask_bits of argus_bn_apply,
 * a block output) and writes part float2[rows][C] = {sum dm, sum dm*(y-mean)*invstd}, rows =
 * argus_conv_dgrad_bn_rows(d, dtype) (C = d->c) — the input of argus_bn_bwd_finalize. Optional second
 * branch (mask_mode 3): y2/mean2/invstd2 -> part2 (the downsample BN of a bottleneck sharing dm).
 * Replaces the ATen batch_norm_backward reduction behind loss.backward() (argus/train.py:316). */
typedef struct {
  const void* y;
  const float* mean;
  const float* invstd;
  int32_t mask_mode;
  int32_t reserved;
  const float* scale;
  const float* shift;
  const uint8_t* mask_bits;
  const void* y2;
  const float* mean2;
  const float* invstd2;
  float* part;
  float* part2;
  /* Optional: with workspace != NULL (argus_bn_workspace_bytes(c), zero-filled once) the BN-backward
   * finalize (argus_bn_bwd_finalize) is folded into the same launch: the last workgroups merge the
   * partials and write dgamma/dbeta (may be NULL) and ca/cb/cc with gamma (+ the second branch). */
  void* workspace;
  const float* gamma;
  float* dgamma;
  float* dbeta;
  float* ca;
  float* cb;
  float* cc;
  const float* gamma2;
  float* dgamma2;
  float* dbeta2;
  float* ca2;
  float* cb2;
  float* cc2;
  /* Optional (ABI 15): with y_x != NULL the main branch's y is not read but recomputed in the kernel as
   * the 1x1 stride-1 convolution of y_x (NHWC, y_k channels, the same pixel grid as dm) with y_w (the
   * bf16 w_fwd copy of that conv, [C][y_k], argus_conv_weight_prep): bit-identical to the y that
   * argus_conv_fwd would have stored, so y itself need not exist (argus_conv_fwd_bn_out with y = NULL).
   * bf16, mask_mode 3, y_k a multiple of 64; y must then be NULL. */
  const void* y_x;
  const void* y_w;
  int32_t y_k;
  int32_t reserved2;
} argus_bn_bwd_epilogue;
/* Optional BN-backward apply folded into the dgrad's operand staging: with `pro` != NULL the `dy`
 * argument of argus_conv_dgrad_bn holds dm (the masked gradient of a BN output) and the dgrad consumes
 * dy = ca*dm + cb*y + cc (per channel; argus_bn_bwd_apply's formula), which it also stores to dy_out
 * for the weight gradient. Kernels that cannot stage it run argus_bn_bwd_apply first (same result).
 * `bn` may be NULL with a prologue: a plain dgrad (no BN-backward epilogue) of the applied dy.
 * dy_out may be NULL when argus_conv_dgrad_stages_prologue(d, dtype) is 1 (1x1 dgrads on the
 * register-staged kernel): dy is then never stored, and the weight gradient stages the same apply
 * from dm itself (argus_conv_wgrad_apply). */
typedef struct {
  const void* y;
  const float* ca;
  const float* cb;
  const float* cc;
  void* dy_out;
} argus_bn_bwd_prologue;
int argus_conv_dgrad_bn_rows(const argus_conv_desc* d, int dtype);
/* 1 when argus_conv_dgrad_bn stages an apply prologue inside the dgrad kernel for this conv (so
 * dy_out may be NULL), 0 when it materialises dy with argus_bn_bwd_apply first. */
int argus_conv_dgrad_stages_prologue(const argus_conv_desc* d, int dtype);
int argus_conv_dgrad_bn(const argus_conv_desc* d, int dtype, const void* dy, const void* w_dgrad,
                        void* dm, const void* addend, const argus_bn_bwd_epilogue* bn,
                        const argus_bn_bwd_prologue* pro, argus_stream_t stream);
/* MX-fp8 stored operands (ABI 16; ARGUS_FP8 networks, the 3x3 stride-1 convs of Bottleneck.conv2 in
 * torchvision's ResNet-50 layers 2-4, argus/models.py:43). An "x8" tensor is the MX-fp8 copy of a bf16
 * NHWC tensor [P][C]: P*C e4m3 bytes (OCP, the value / 2^e rounded to nearest even) followed by P*C/32
 * E8M0 scale bytes (127 + e, one per 32 consecutive channels of a pixel), e chosen as ARGUS_FP8's
 * staging quantizer chooses it; argus_bn_apply_x8 / argus_bn_bwd_apply_x8 write it beside their bf16
 * output. argus_conv_fwd_x8 is argus_conv_fwd(ARGUS_FP8) without a prologue, its input read as the x8
 * copy x8 (bit-identical to quantizing the bf16 input while staging); argus_conv_dgrad_bn_x8 is
 * argus_conv_dgrad_bn(ARGUS_FP8) with dy read as x8 (bn NULL, or mask mode 2; no addend / prologue /
 * y recompute). Both need the fp8 weight copies of argus_conv_weight_prep(ARGUS_FP8): policy key 37
 * bit 8 (forward of 3x3 stride-1 convs) and bit 2 (3x3 data gradients). argus_conv_x8_ok(d, pass)
 * is 1 when pass 0 (forward) / 1 (data gradient) of d is served (C resp. K % 128 == 0, the LDS-halo
 * shapes, the policy bits). */
int argus_conv_x8_ok(const argus_conv_desc* d, int pass);
int argus_conv_fwd_x8(const argus_conv_desc* d, const void* x8, const void* w_fwd, void* y, float* stat_part,
                      argus_stream_t stream);
int argus_conv_dgrad_bn_x8(const argus_conv_desc* d, const void* dy8, const void* w_dgrad, void* dm,
                           const argus_bn_bwd_epilogue* bn, argus_stream_t stream);
/* Kernel-selection policy: the library's immutable default of a key (-1 for an unknown key); a conv
 * descriptor may override keys for its own call (argus_conv_desc.tuning; an unknown key there makes
 * the call fail with ARGUS_ERR_ARG). Every default is the measured best.
 * key 0..2 force the row tile (64|128, 0 = heuristic) of pass fwd/dgrad/wgrad, key 3..5 the column
 * tile, key 6 the wgrad split target (workgroups), key 7 the largest K (= taps*C) served by the
 * 4-workgroups-per-CU single-buffer forward/dgrad kernel, key 8 the smallest K served by the bf16
 * global->LDS (glds) forward/dgrad kernel (0 disables it), key 9 the fewest workgroups for which
 * that kernel is chosen, key 10 enables (1) or disables (0) the LDS-halo kernel for 3x3 stride-1
 * forward/dgrad, key 11 the same for the 3x3 stride-1 weight gradient and key 12 its split target,
 * key 13 the fewest workgroups for the fwd/dgrad halo kernel (1 also allows its 64-channel variant
 * at any size), key 14 the most (64 x 64) channel tiles for the wgrad halo kernel, key 19 the bf16
 * stem forward on the LDS-patch kernel (1) or the implicit GEMM (0), key 27 the split target of the
 * register-staged 3x3 weight gradient, key 34 the bf16 stem weight gradient on the LDS-patch kernel
 * (1) or on the register-staged weight-gradient kernel (0), key 35 the fewest GEMM rows (output
 * pixels) for which the forward uses 128-row tiles (fewer: 64), key 36 the fewest GEMM rows for the
 * glds kernel, key 37 which ARGUS_FP8 passes take MX-fp8 operands (bits: 1 forward, 2 data gradient of
 * a 3x3 conv, 4 data gradient of a 1x1 conv, 8 forward of a 3x3 stride-1 conv; default 10;
 * argus_conv_weight_prep follows the same key), key 42 the
 * workgroups per CU (4 or 3) the small-K BN-epilogue / apply-prologue data gradients are built for,
 * key 43 the bottleneck conv1 data gradients on the persistent kernel (1) or the igemm (0), key 44 the
 * statistics-only 1x1 forwards on the persistent kernel (1) or the igemm (0), key 45 the 1x1 bf16
 * weight gradients on the LDS-DMA ring kernel with 128 x 128 tiles (1), 128 x 256 tiles where
 * Cin % 256 == 0 for the BN-backward-apply form (2) or both forms (3), or the register-staged one (0);
 * key 46 the pixel count up to which 1x1 weight gradients take half the split target (key 6); key 47
 * the stride-2 plain bf16 weight gradients (1x1, 3x3) on the DMA kernel with gathered x rows (1) or not (0).
 * (Keys scaled with the batch keep a smaller batch's kernel selection that of the larger one:
 * tests/test_gpu_parity.py stage-checks the benched configurations' kernels that way.) */
int argus_conv_policy_default(int key);
/* Which tile a pass launches and its algorithmic work: pass 0 fwd, 1 dgrad, 2 wgrad. Returns a
 * tag (kind*10^7 + dtype*10^6 + tile_m*1000 + tile_n; kind 1 igemm, 2 wgrad) and writes
 * 2*P*K*R*S*C flops (P = n*ho*wo output pixels). */
int argus_conv_launch_info(const argus_conv_desc* d, int dtype, int pass, int64_t* flops);
/* dw (fp32, OHWI 7x7x3 for the stem) = sum over pixels of dy x im2col(x'), x' as in conv_fwd. */
size_t argus_conv_wgrad_workspace_bytes(const argus_conv_desc* d, int dtype);
int argus_conv_wgrad(const argus_conv_desc* d, int dtype, const void* x, const float* pro_scale,
                     const float* pro_shift, const void* dy, float* dw, void* workspace,
                     size_t workspace_bytes, argus_stream_t stream);
/* Weight gradient whose dy = ca*dm + cb*y + cc (BN-backward apply, argus_bn_bwd_apply's formula) is
 * formed while staging its operand from dm (ap->dy_out is ignored): dy is never materialised. Used
 * for the stem (whose dy feeds nothing else) and for the 1x1 convs whose dgrad stages the same apply
 * (argus_conv_dgrad_stages_prologue). Runs the register-staged wgrad kernel; the input x has no
 * BN prologue. */
int argus_conv_wgrad_apply(const argus_conv_desc* d, int dtype, const void* x, const void* dm,
                           const argus_bn_bwd_prologue* ap, float* dw, void* workspace,
                           size_t workspace_bytes, argus_stream_t stream);
/* Data and weight gradient of one 1x1 stride-1 conv in one pass over its output gradient (torch's
 * convolution backward with output_mask (grad_input, grad_weight) for Bottleneck.conv3 of ResNet-50
 * layer 1 and of the first block's downsample, reached from loss.backward() at argus/train.py:316;
 * replaces argus_conv_dgrad_bn (argus_conv_dgrad) +
 * argus_conv_wgrad_apply for that conv). `dm`, `pro` as in argus_conv_dgrad_bn with an apply
 * prologue (pro->dy_out must be NULL: dy is never stored); `bn` a mask-mode-2 BN-backward epilogue
 * (its partial rows: argus_conv_dgrad_wgrad_bn_rows; with bn->workspace the finalize is folded), or
 * NULL for a plain dx, optionally dx += addend (may alias dx; the first block's downsample);
 * x = the conv input (for dw, fp32 OHWI). bf16 only, C = 64 input and K = 256 output channels
 * (argus_conv_dgrad_wgrad_ok); workspace: argus_conv_dgrad_wgrad_workspace_bytes. */
int argus_conv_dgrad_wgrad_ok(const argus_conv_desc* d, int dtype);
size_t argus_conv_dgrad_wgrad_workspace_bytes(const argus_conv_desc* d, int dtype);
int argus_conv_dgrad_wgrad_bn_rows(const argus_conv_desc* d, int dtype);
int argus_conv_dgrad_wgrad_bn(const argus_conv_desc* d, int dtype, const void* dm, const void* w_dgrad,
                              const void* x, void* dx, const void* addend, const argus_bn_bwd_epilogue* bn,
                              const argus_bn_bwd_prologue* pro, float* dw, void* workspace,
                              size_t workspace_bytes, argus_stream_t stream);

/* ---- kernel timer (bench.py roofline) ------------------------------------------------------------
 * While enabled, conv and BN kernel launches whose demangled instantiation name (e.g.
 * "argus::igemm_kernel<__bf16, 128, 128, false, true>", as c++filt prints rocprofv3's kernel name)
 * starts with `filter` (NULL or "" = all) are dispatched with hipExtLaunchKernelGGL start/stop
 * events, i.e. timed by the dispatch packet on the launch stream. enable() clears old records;
 * count() synchronizes the recorded events, aggregates per name and returns the number of names;
 * get(i) returns name, launches, total milliseconds, total algorithmic flops (0 for BN kernels) and
 * total algorithmic HBM bytes (each operand read once and each result written once; for wgrad the
 * fp32 split partials it writes count too). */
int argus_ktimer_enable(const char* filter);
/* argus_ktimer_enable restricted to launches on `stream` (e.g. the caller's main stream: the
 * critical path of a step whose weight gradients run on a side stream). */
int argus_ktimer_enable_on(const char* filter, argus_stream_t stream);
int argus_ktimer_disable(void);
int argus_ktimer_count(void);
int argus_ktimer_get(int index, char* name, int name_len, int64_t* launches, double* total_ms,
                     double* work, double* bytes);

/* ---- cross-stream ordering (ABI 19) ------------------------------------------------------------
 * Events for ordering two streams of one device: created with hipEventDisableTiming |
 * hipEventDisableSystemFence, so recording one performs a device-scope release and waiting on it a
 * device-scope acquire, without the system-scope cache writeback / invalidation a default event carries.
 * Work on this device only (the weight-gradient side stream and the main stream of one process); the
 * host and other devices need a default event. Replaces the torch.cuda.Event record / wait_event pairs
 * the DDP-free training step of argus/train.py:298-321 would use between two streams (it uses one). */
typedef void* argus_event_t; /* hipEvent_t */
int argus_event_create(argus_event_t* event);
int argus_event_record(argus_event_t event, argus_stream_t stream);
int argus_stream_wait_event(argus_stream_t stream, argus_event_t event);
int argus_event_destroy(argus_event_t event);

/* ---- BatchNorm2d (train: batch stats, eps, momentum; eval: running stats) --------------------- */
/* Workspace of argus_bn_finalize / argus_bn_bwd_finalize / the folded finalize of argus_conv_dgrad_bn
 * for up to `channels` channels. Its first 16 KiB hold inter-workgroup ticket counters: zero-fill the workspace ONCE when it is allocated;
 * the kernels leave the counters zero (do not share one workspace between concurrent streams). */
size_t argus_bn_workspace_bytes(int channels);
/* From tile partials float2[rows][C] = {sum, M2 (sum of squared deviations from the tile mean)},
 * tile t holding min(tile_rows, count - t*tile_rows) elements per channel (as argus_conv_fwd
 * writes them; tile_rows < 0, as argus_conv_fwd_stat_tile reports for a producer with ragged tiles:
 * row r holds counts[r] <= |tile_rows| elements, the int32 counts[rows] stored right after the
 * float2[rows][C] partials, i.e. at (const int*)(part + 2*rows*C)): merged
 * in fp64 (Chan), gives mean, invstd, the fused apply coefficients
 * scale = gamma*invstd, shift = beta - mean*scale; updates running stats (momentum, unbiased
 * variance) and num_batches_tracked when those pointers are non-NULL. */
int argus_bn_finalize(int channels, int rows, int tile_rows, const float* part, int64_t count,
                      const float* gamma,
                      const float* beta, float eps, float momentum, float* running_mean,
                      float* running_var, int64_t* num_batches_tracked, float* mean, float* invstd,
                      float* scale, float* shift, void* workspace, argus_stream_t stream);
int argus_bn_eval_coeffs(int channels, const float* gamma, const float* beta,
                         const float* running_mean, const float* running_var, float eps,
                         float* scale, float* shift, argus_stream_t stream);
/* out = [relu]( y*scale+shift + residual' ), residual' = res*res_scale+res_shift (if res_scale),
 * res (if res), else 0. out may alias y. If mask_out != NULL it also receives the ReLU mask of out:
 * one byte per 16-byte chunk (8 bf16 / 4 fp32 channels), bit j set <=> element j of the chunk > 0,
 * i.e. mask_out[(pixel*channels + c) / E] bit (c % E). */
int argus_bn_apply(int dtype, int64_t pixels, int channels, const void* y, const float* scale,
                   const float* shift, const void* res, const float* res_scale,
                   const float* res_shift, int relu, void* out, uint8_t* mask_out,
                   argus_stream_t stream);
/* argus_bn_apply (bf16, channels % 32 == 0) that also writes the x8 copy of out to out8 (ABI 16;
 * argus_conv_fwd_x8). */
int argus_bn_apply_x8(int64_t pixels, int channels, const void* y, const float* scale, const float* shift,
                      const void* res, const float* res_scale, const float* res_shift, int relu, void* out,
                      uint8_t* mask_out, void* out8, argus_stream_t stream);
/* Backward. mask_mode: 0 none; 1 relu mask from the tensor `mask` (>0, e.g. a block output);
 * 2 relu mask recomputed from y as (y*scale+shift > 0); 3 relu mask from the bits `mask` written
 * by argus_bn_apply. dm = dz*mask.
 * reduce: part float2[rows][C] = {sum dm, sum dm*(y-mean)*invstd}; rows = argus_bn_bwd_rows().
 * Optional second branch (y2 != NULL; modes 0/1/3): a second BN whose output was summed with the
 * first before the same ReLU (bn3 + the downsample BN of a bottleneck) shares dm, so both are
 * reduced / applied in one pass: part2 = {sum dm, sum dm*(y2-mean2)*invstd2}, dy2 = ca2*dm + cb2*y2 + cc2. */
int argus_bn_bwd_rows(int64_t pixels, int channels);
int argus_bn_bwd_reduce(int dtype, int64_t pixels, int channels, const void* dz, int mask_mode,
                        const void* mask, const void* y, const float* scale,
                        const float* shift, const float* mean, const float* invstd, float* part,
                        const void* y2, const float* mean2, const float* invstd2, float* part2,
                        argus_stream_t stream);
/* dgamma/dbeta (fp32, written) and coefficients so that dy = ca*dm + cb*y + cc. */
int argus_bn_bwd_finalize(int channels, int rows, const float* part, int64_t count,
                          const float* gamma, const float* mean, const float* invstd,
                          float* dgamma, float* dbeta, float* ca, float* cb, float* cc,
                          void* workspace, argus_stream_t stream);
/* dy = ca*dm + cb*y + cc (dtype); if dm_out != NULL also writes dm (the masked dz). */
int argus_bn_bwd_apply(int dtype, int64_t pixels, int channels, const void* dz, int mask_mode,
                       const void* mask, const void* y, const float* scale, const float* shift,
                       const float* ca, const float* cb, const float* cc, void* dy, void* dm_out,
                       const void* y2, const float* ca2, const float* cb2, const float* cc2, void* dy2,
                       argus_stream_t stream);
/* dy = ca*dm + cb*y + cc from an already-masked dm (mask mode 0, bf16, channels % 32 == 0), plus the
 * x8 copy of dy in dy8 (ABI 16; argus_conv_dgrad_bn_x8). */
int argus_bn_bwd_apply_x8(int64_t pixels, int channels, const void* dm, const void* y, const float* ca,
                          const float* cb, const float* cc, void* dy, void* dy8, argus_stream_t stream);

/* ---- pooling (MaxPool2d(3,2,1) fused with the stem's BN+ReLU; AdaptiveAvgPool2d(1)) ----------- */
int argus_maxpool_fwd(int dtype, int n, int h, int w, int c, const void* y, const float* scale,
                      const float* shift, void* out, uint8_t* argmax, argus_stream_t stream);
int argus_maxpool_bwd(int dtype, int n, int h, int w, int c, const void* dout,
                      const uint8_t* argmax, void* dz, argus_stream_t stream);
/* maxpool backward with the stem BatchNorm's backward reduction fused (the pooled tensor is
 * relu(y*scale+shift), y the stem conv output): stores dm = dz * (y*scale+shift > 0) and
 * part float2[argus_maxpool_bwd_bn_rows()][c] = {sum dm, sum dm*(y-mean)*invstd}, the input of
 * argus_bn_bwd_finalize. y == NULL: plain argus_maxpool_bwd. */
int argus_maxpool_bwd_bn_rows(int dtype, int n, int h, int w, int c);
int argus_maxpool_bwd_bn(int dtype, int n, int h, int w, int c, const void* dout, const uint8_t* argmax,
                         void* dm, const void* y, const float* scale, const float* shift,
                         const float* mean, const float* invstd, float* part, argus_stream_t stream);
/* argus_maxpool_bwd_bn with argus_bn_bwd_finalize folded in (ABI 13; c % 64 == 0): the last workgroups
 * of the pass merge `part` (write-through, deterministic fixed order) and write dgamma/dbeta (may be
 * NULL) and ca/cb/cc exactly as argus_bn_bwd_finalize(c, rows, part, n*h*w, gamma, mean, invstd, ...)
 * would; `workspace` is an argus_bn_workspace_bytes(c) BN workspace (zeroed once, not shared between
 * concurrent streams). workspace == NULL: argus_maxpool_bwd_bn. Backward of the torchvision stem
 * bn1 -> relu -> maxpool inside self.resnet(x) (models.py:43,84) under loss.backward() (train.py:316). */
int argus_maxpool_bwd_bn_fin(int dtype, int n, int h, int w, int c, const void* dout, const uint8_t* argmax,
                             void* dm, const void* y, const float* scale, const float* shift,
                             const float* mean, const float* invstd, float* part, const float* gamma,
                             float* dgamma, float* dbeta, float* ca, float* cb, float* cc, void* workspace,
                             argus_stream_t stream);
int argus_avgpool_fwd(int dtype, int n, int hw, int c, const void* x, float* feat,
                      argus_stream_t stream);
int argus_avgpool_bwd(int dtype, int n, int hw, int c, const float* dfeat, void* dx,
                      argus_stream_t stream);

/* ---- FC / MLP head (nn.Linear + exact GELU; models.py:56-64,88), fp32 ------------------------ */
/* C[m][n] = sum_k opA(A)[m][k] * opB(B)[k][n]; opA(A)[m][k] = trans_a ? A[k*lda+m] : A[m*lda+k],
 * opB(B)[k][n] = trans_b ? B[n*ldb+k] : B[k*ldb+n].
 * epilogue 0: C = acc; 1: C = acc + bias[n]; 2: aux = acc + bias[n], C = gelu(aux);
 * 3: C = acc * gelu'(aux[m][n]) (backward through a GELU whose pre-activation is aux, ld = ldc);
 * 4: C += acc. Small-output / long-K products split K over workgroups (deterministic fixed-order
 * reduce) when a workspace of argus_gemm_f32_workspace_bytes() is given (NULL: no split). */
size_t argus_gemm_f32_workspace_bytes(int m, int n, int k);
int argus_gemm_f32(int m, int n, int k, const float* a, int lda, int trans_a, const float* b,
                   int ldb, int trans_b, float* c, int ldc, const float* bias, int epilogue,
                   float* aux, void* workspace, size_t workspace_bytes, argus_stream_t stream);
/* out[n] = sum_m x[m*ld + n] (bias gradients). */
int argus_colsum_f32(int m, int n, const float* x, int ld, float* out, argus_stream_t stream);
int argus_gelu_f32(int64_t count, const float* x, float* y, argus_stream_t stream);
int argus_gelu_bwd_f32(int64_t count, const float* x, const float* dy, float* dx,
                       argus_stream_t stream);

/* ---- SE(3) geodesic loss (geometric_loss_fn, argus/train.py:105-119; pypose Exp/Inv/@/Log) ---- */
/* loss[b] = |Log(Exp(pred_b) @ target_b^-1)|^2 ; dpred[b] = grad_scale * d loss[b] / d pred[b]
 * (dpred may be NULL). pred (B,6) [rho, phi]; target (B,7) [t, qx, qy, qz, qw]. */
int argus_se3_loss(int batch, const float* pred, const float* target, float* loss, float* dpred,
                   float grad_scale, argus_stream_t stream);

/* se(3) -> SE(3) exponential (pypose se3.Exp; get_pose, argus/utils.py:179-189): out (B,7) =
 * [t, qx, qy, qz, qw]; canonical_w != 0 flips q to w >= 0. */
int argus_se3_exp(int batch, const float* xi, float* out, int canonical_w, argus_stream_t stream);

/* ---- photometric training augmentations (argus/data.py:41-103; csrc/augment.hip) -------------
 * src: uint8 images (n_img, 3, H, W) planar (a B x 6 x H x W sample batch is 2B such images);
 * dst: fp32 (same shape) = augmented src / 255; params: n_img AugParams records of
 * argus_augment_params_bytes() bytes each (device memory; layout in augment.hip / augment.py);
 * scratch: argus_augment_scratch_bytes() bytes. Random erasing (two rectangles) -> Planckian gains
 * -> ColorJiggle (sampled op order) -> 5x5 Gaussian blur (reflect) -> 3x3 motion blur (zero border)
 * -> plasma shadow (diamond-square map) -> salt-and-pepper, per image. */
size_t argus_augment_params_bytes(void);
size_t argus_augment_scratch_bytes(int64_t n_img, int h, int w);
int argus_augment_photometric(int64_t n_img, int h, int w, const uint8_t* src, float* dst, const void* params,
                              float* scratch, argus_stream_t stream);

/* ---- optimizer step (clip_grad_norm_ + Adam, argus/train.py:232,317-320) --------------------- */
size_t argus_sumsq_workspace_bytes(int64_t count);
/* out[0] = sqrt(sum x^2) (fp32, deterministic two-level reduction). */
int argus_global_norm(int64_t count, const float* x, float* out, void* workspace,
                      argus_stream_t stream);
/* g' = grad_scale*g (e.g. 1/world after a SUM all-reduce); if norm != NULL (norm[0] = |g|),
 * g' *= min(1, max_norm/(grad_scale*norm[0]+1e-6)) (clip_grad_norm_); then Adam (torch
 * semantics, bias corrections bc1 = 1-beta1^t, bc2 = 1-beta2^t); writes param, m, v. */
int argus_adam_step(int64_t count, float* param, const float* grad, float* exp_avg,
                    float* exp_avg_sq, const float* norm, float grad_scale, float max_norm,
                    float lr, float beta1, float beta2, float eps, float weight_decay, float bc1,
                    float bc2, argus_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ARGUS_HIP_H */
