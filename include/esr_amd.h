/*
 * esr_amd.h — C ABI of the MI355X-native RRDB-23 + CEM ×4 super-resolution hot path (libesr_amd.so).
 *
 * Every entry point is `extern "C"`, takes plain pointers / sizes, enqueues on the given HIP stream and returns 0 or a
 * negative esr_status.  Buffers are caller-allocated device memory; the library holds no persistent allocations and no
 * mutable selection state — which kernel a launch runs is a function of its arguments only — so every entry point is
 * stateless and re-entrant across streams and threads.  The kernel-selection switches used for A/B
 * measurements live only in the separate ablation build (csrc/esr_ablation.h, `make exp`).
 *
 * Reference = YuvalBahat/Explorable-Super-Resolution_old, paths relative to codes/.  Each entry cites the reference
 * interface it replaces.  The Python host layer (explorable-super-resolution_old_amd/esr_amd) binds these through
 * ctypes behind the reference's RRDBNet / CEM_PyTorch / define_G API.
 *
 * Feature-map layout ("padded NHWC"): fp32 [B][H+2][W+2][cp], a one-pixel zero halo around the H×W interior, `cp`
 * floats per pixel (channel pitch, multiple of 4).  Interior pixel (b, y, x), channel c lives at
 *     ((b*(H+2) + y+1)*(W+2) + x+1)*cp + c.
 * A convolution reads the channel PREFIX [0, cin) of its input pixels, which is how the dense concatenations of the
 * residual dense block (block.py:233-235) are realised without copies: each conv writes its growth channels into a
 * slice of the same buffer.
 */
#ifndef ESR_AMD_H
#define ESR_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *esr_stream_t; /* hipStream_t (0 = legacy default stream) */

enum esr_status {
    ESR_OK = 0,
    ESR_EINVAL = -1,   /* bad shape / alignment / unsupported combination */
    ESR_ELAUNCH = -2,  /* kernel launch failed (hipGetLastError after launch) */
};

/* Packed conv weights: [nchunk][taps][n_pad][32] fp32, nchunk = ceil(cin/32), n_pad = 32*ceil(cout/32); channel c of
 * chunk j is input channel 32*j + c (zero where >= cin).  Bias: fp32 [cout]. */

/* Output/epilogue descriptor of a convolution.
 *   v = acc + bias[n]; if (lrelu == 1) v = v > 0 ? v : 0.2*v   (conv_block CNA + act, block.py:10-23,141-146)
 *   if (r1) v = s1*v + r1[pixel, r1_coff + n]                  (RDB / trunk residuals, block.py:96,235,270)
 *   if (lrelu == 2) v = r2[pixel, r2_coff + n] > 0 ? v : 0.2*v (LeakyReLU backward through the saved activation r2;
 *                                                               r2 required; lrelu == 3: r2 in the split-f16
 *                                                               layout, r2_cp/r2_coff % 8 == 0; the x3 convs take
 *                                                               lrelu 0, 1 and 3)
 *   else if (r2) v = s2*v + r2[pixel, r2_coff + n]
 *   out[pixel, out_coff + n] = v   (and out2 likewise when out2 != NULL)
 * Output pixel of input-grid position (y, x) is (out_sy*y + out_oy, out_sx*x + out_ox) in the out grid (out_h × out_w,
 * padded NHWC), which is how the four polyphase phases of the nearest-×2 upconv scatter into the 2× grid.
 * out_planar = 1 writes NCHW [B][cout][out_h][out_w] without halo instead (the generator output fed to CEM).
 * r1/r2/out2 use the out grid geometry with their own channel pitch/offset. */
typedef struct esr_conv_out {
    float *out;
    int32_t out_cp, out_coff, out_h, out_w, out_sy, out_sx, out_oy, out_ox, out_planar;
    int32_t lrelu;
    const float *r1;
    int32_t r1_cp, r1_coff;
    float s1;
    const float *r2;
    int32_t r2_cp, r2_coff;
    float s2;
    float *out2;
    int32_t out2_cp, out2_coff;
} esr_conv_out;

/* 3×3 stride-1 zero-pad-1 convolution + bias + LeakyReLU/residual epilogue, fp32 (f32-input MFMA, exact fp32 FMA
 * chain).  Replaces nn.Conv2d(k=3, padding=1) + act in conv_block (block.py:129-156), i.e. every generator conv of
 * RRDBNet (architecture.py:122-141): conv_first, the 345 RDB convs (block.py:212-217), LR_conv, HR_conv0/1.
 * in: padded NHWC [B][H+2][W+2][in_cp], reads channels [0, cin); cin % 8 == 0; cout <= 64. */
int esr_conv3x3_fwd(const float *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                    const float *w_packed, const float *bias, int32_t cout, const esr_conv_out *o, esr_stream_t stream);

/* One polyphase phase (py, px) in {0,1}² of the nearest-×2 upsample + 3×3 conv (upconv_blcok, block.py:294-301;
 * used twice by RRDBNet, networks.py:91): out[2y+py, 2x+px] = Σ_{a,b∈{0,1}} Wp[a][b] · in[y+py+a-1, x+px+b-1], with
 * Wp the 3×3 taps summed per source pixel (folded on the host, see esr_amd/ops.py).  w_packed: [nchunk][4][n_pad][32].
 * Set o->out_sy = o->out_sx = 2, o->out_oy = py, o->out_ox = px. */
int esr_upconv2x_phase_fwd(const float *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                           const float *w_packed, const float *bias, int32_t cout, int32_t py, int32_t px,
                           const esr_conv_out *o, esr_stream_t stream);

/* Model-input preparation (SRRaGANModel.ConcatLatent SRRaGAN_model.py:249-255, CEM_PyTorch pre-pad CEMnet.py:170-181,
 * RRDBNet latent split + bilinear ↓sf architecture.py:153-160).
 * x: NCHW fp32 [B][nz*sf*sf + 3][h][w] (nz = 0 plain, 3 latent; the HR latent travels as a raw view).
 * Writes, for the padded LR grid H = h+2m, W = w+2m (m = pre-pad margin, 0 in train mode), replicate padding:
 *   lr_nchw  [B][3][H][W]                   padded LR image (CEM input, CEMnet.py:184)
 *   first    padded NHWC [B][H+2][W+2][first_cp]: Z_LR at channels 0..nz-1, LR at channels first_lr_off..+2
 *   zlr_dst[i] padded NHWC LR-grid buffers with their own pitch zlr_cp[i]: Z_LR at channels 0..nz-1 (i < n_zlr)
 *   zhr_dst[i] padded NHWC HR-grid buffers (sf*H × sf*W), pitch zhr_cp[i]: Z_HR (replicate pad sf*m) at 0..nz-1
 * Z_LR = F.interpolate(Z_HR_padded, 1/sf, bilinear, align_corners=False).
 * split = 1 writes `first` and the Z slots in the split-f16 layout of the x3 path (below), 0 in fp32. */
int esr_prep_input(const float *x, int32_t B, int32_t nz, int32_t h, int32_t w, int32_t sf, int32_t m,
                   float *lr_nchw, float *first, int32_t first_cp, int32_t first_lr_off,
                   float *const *zlr_dst, const int32_t *zlr_cp, int32_t n_zlr,
                   float *const *zhr_dst, const int32_t *zhr_cp, int32_t n_zhr, int32_t split, esr_stream_t stream);
/* esr_prep_input with the split outputs (split = 1) written as v × act_scale, a power of two (the x3 forward's
 * activation scale: every split activation of an x3 forward holds A·v, so that small activations keep their f16 lo
 * parts in the normal range; the x3 convs carry it through with their biases scaled by A and the planar HR_conv1 output
 * divided by it).  The fp32 LR copy for CEM (lr_nchw) is never scaled. */
int esr_prep_input_s(const float *x, int32_t B, int32_t nz, int32_t h, int32_t w, int32_t sf, int32_t m,
                     float *lr_nchw, float *first, int32_t first_cp, int32_t first_lr_off, float *const *zlr_dst,
                     const int32_t *zlr_cp, int32_t n_zlr, float *const *zhr_dst, const int32_t *zhr_cp,
                     int32_t n_zhr, int32_t split, float act_scale, esr_stream_t stream);

/* CEM step 1, fused DownscaleOP + LR residual (CEMnet.py:152,157-162,186-189):
 *   r[b,c,i,j] = (lr ? lr[b,c,i,j] : 0) - Σ_{u,v<kd} w_down[u][v] · gen[b,c, clamp(sf*i+ph+u-kd/2), clamp(sf*j+ph+v-kd/2)]
 * gen: NCHW [B][3][sf*H][sf*W]; lr, r: NCHW [B][3][H][W]; w_down = rot180(ds_kernel) (the Filter_OP weight),
 * kd odd; ph = the stride phase (calc_strides pre_stride, imresize_CEM.py:83-85).  With lr == NULL this is
 * -DownscaleOP(gen) (GUI.py:1289,1900 use DownscaleOP alone; pass negate=1 to get +DownscaleOP). */
int esr_cem_down(const float *gen, const float *lr, float *r, int32_t B, int32_t H, int32_t W, int32_t sf, int32_t ph,
                 const float *w_down, int32_t kd, int32_t negate, esr_stream_t stream);

/* CEM step 2, Conv_LR_with_Inv_hTh_OP (CEMnet.py:149-151): q = xcorr(replicate_pad(r, ki/2), w_inv), NCHW LR grid,
 * C = 3 channels, ki odd. */
int esr_cem_inv(const float *r, float *q, int32_t B, int32_t H, int32_t W, const float *w_inv, int32_t ki,
                esr_stream_t stream);

/* CEM step 3, Upscale_OP + back-projection + HR unpad (CEMnet.py:153-159,186-190):
 *   out[b,c,Y,X] = gen[b,c,Y+M,X+M] + Σ_{u,v<kd} w_up[u][v] · S[clamp(Y+M+u-kd/2), clamp(X+M+v-kd/2)]
 * S = q zero-stuffed at phase ph on the sf× grid; M = HR crop margin (0 in train mode).
 * out: NCHW [B][3][sf*H-2M][sf*W-2M]; w_up = sf²·ds_kernel. */
int esr_cem_up_add(const float *q, const float *gen, float *out, int32_t B, int32_t H, int32_t W, int32_t sf,
                   int32_t ph, const float *w_up, int32_t kd, int32_t M, esr_stream_t stream);

/* ---- split-precision ("x3") path --------------------------------------------------------------------------------
 * Split activation layout: padded NHWC as above, 4 bytes per channel, channels in groups of 8; group g of a pixel is
 * 32 bytes: f16 hi[8] then f16 lo[8] with hi = f16(v), lo = f16(v - hi) (|v - hi - lo| <= 2^-22 |v|).  cp, cin and
 * every channel offset are multiples of 8.  Packed x3 weights: [nchunk16][taps][n_pad][16 channels as 2 split groups]
 * (64 B per (tap, n)), scaled by `w_scale` (a power of two the epilogue divides out exactly).
 * Products are a_hi·b_hi + a_hi·b_lo + a_lo·b_hi on v_mfma_f32_32x32x16_f16 with fp32 accumulation.
 * Outputs are split unless o->out_planar (fp32 NCHW).  r1/r2 residual inputs are split.  *overflow is OR-ed with 1
 * if any split output is not representable (|v| >= 65504), in which case the caller reruns the exact-fp32 path.
 * Kernel choice (a function of the shape): the column-tile kernel (esr_conv_x3c.hip; 12-column tiles at three
 * workgroups per CU for cout <= 32, an N = 64 conv on a grid that cannot give every CU two workgroups as two N = 32
 * launches over the halves of its weights) or, for small N = 32 grids, the classic 8-row kernel at three workgroups per
 * CU; a 3×3 conv with cout <= 3, cin <= 80 and a planar output without residuals (HR_conv1) on the narrow-N kernel (the
 * 9 taps × 3 outputs in the MFMA M dimension).  All are bitwise identical except the narrow-N kernel (tap sums in
 * another order).  Blocks map to tiles in XCD-grouped order. */
int esr_conv3x3_fwd_x3(const void *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                       const void *w_packed, const float *bias, float w_scale, int32_t cout, const esr_conv_out *o,
                       int32_t *overflow, esr_stream_t stream);
int esr_upconv2x_phase_fwd_x3(const void *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                              const void *w_packed, const float *bias, float w_scale, int32_t cout, int32_t py,
                              int32_t px, const esr_conv_out *o, int32_t *overflow, esr_stream_t stream);

/* HR_conv0 + LeakyReLU and HR_conv1 of RRDBNet (architecture.py:140-141, 172-174) in the x3 inference forward,
 * without HR_conv0's activations ever reaching memory (replaces esr_conv3x3_fwd_x3 of HR_conv0 into a split buffer
 * followed by HR_conv1's narrow-N launch, which re-read that 4 B/channel buffer).
 * esr_hr_convs_x3: the HR_conv0 conv (in: the split HR-grid buffer, in_cp = zc + 64 channels = [latent slot of zc
 * channels (0 or 8, prep_hr's Z) | 64 upsampled features]; w0/bias0/w0_scale as esr_conv3x3_fwd_x3 with cout 64) whose
 * epilogue computes, per interior pixel p, y[p][3t + o] = Σ_c W1[o][c][t] · a[p][c] for HR_conv1's 9 taps t and 3
 * outputs o over its input a = [the latent slot of `in` | lrelu(HR_conv0)] (w1: HR_conv1's x3-packed weights, n_pad
 * 32, scaled like any x3 weight; x3 products on the matrix cores).  y: padded [B][H+2][W+2][32] fp32 (27 used), 16-B
 * aligned, halo zero (never written).  *overflow |= 1 if an activation is not representable in f16 (as a split store).
 * esr_hr1_sum: out NCHW [B][3][H][W] = scale_inv · Σ_{ty,tx} y[b][y+ty][x+tx][3(3ty+tx) + o] + bias1[o]
 * (scale_inv = 1/(w1_scale · activation scale)).  Equal to the unfused pair up to the summation order. */
int esr_hr_convs_x3(const void *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t zc, const void *w0,
                    const float *bias0, float w0_scale, const void *w1, float *y, int32_t *overflow,
                    esr_stream_t stream);
int esr_hr1_sum(const float *y, int32_t B, int32_t H, int32_t W, const float *bias1, float scale_inv, float *out,
                esr_stream_t stream);

/* ---- training / Z-optimisation backward (esr_train.hip) ------------------------------------------------------------
 * The data gradient of every conv is esr_conv3x3_fwd run with rot180, in/out-swapped packed weights (host-side
 * repacking), i.e. the backward of conv_block (block.py:129-156) for loss.backward() in
 * SRRaGANModel.optimize_parameters (SRRaGAN_model.py:529) and Z_optimizer.optimize (Z_optimization.py:633). */

/* Weight + bias gradient of a 3×3 zero-padded conv on the H×W output grid:
 *   partial[s][tap][ci][co] = Σ_{pixels of split s} in[p + tap][ci] · dout[p][co],   partial[s][9*cin_pad*cout_pad + co]
 *   = Σ dout[p][co] (bias), cin_pad = 32·ceil(cin/32), cout_pad = 32·ceil(cout/32).
 * in: padded NHWC fp32, channels [0, cin) (cin % 4 == 0); flags bit 0 (up2): the conv input is the nearest-×2
 * upsampling of an (H/2)×(W/2) `in` grid (the upconv of block.py:294-301); flags bit 1: `in` is in the split-f16
 * layout (the x3 forward's activations; cin, in_cp % 8 == 0; 12-wave kernel only).  dout: padded NHWC fp32 on the
 * H×W grid, channels [dout_coff, dout_coff + cout), cout <= 64.  Deterministic: reduce the `splits` partials with
 * esr_wgrad_reduce. */
int esr_conv3x3_wgrad(const float *in, int32_t in_cp, int32_t cin, int32_t flags, const float *dout, int32_t dout_cp,
                      int32_t dout_coff, int32_t cout, int32_t B, int32_t H, int32_t W, int32_t splits, float *partial,
                      esr_stream_t stream);
/* out[i] = scale · Σ_s partial[s·n + i], fixed summation order. */
int esr_wgrad_reduce(const float *partial, int32_t splits, int64_t n, float scale, float *out, esr_stream_t stream);

/* ---- x3 backward (split-f16 gradients) ----------------------------------------------------------------------------
 * esr_conv3x3_wgrad flags: bit 0 = nearest-×2 input (upconv), bit 1 = input in the split-f16 layout (the x3 forward's
 * activations), bit 2 = x3 products on f16 MFMA (requires bit 1; the output gradient is split per pixel tile after
 * a power-of-two scaling chosen from the tile's max, the accumulators rescaled exactly between tiles), bit 3 = the
 * output gradient itself in the split layout (requires bit 2; cout, dout_cp, dout_coff % 8 == 0).
 * Inside the residual blocks the x3 backward keeps its data gradients in the split layout, scaled by a power of two
 * S per RRDB so that they sit inside f16's range: S = 2^(11 - ex) for max|g| < 2^ex, g the fp32 trunk gradient at
 * the block's output, whose max esr_grad_amax accumulates (as float bits, atomic max) into *amax (zeroed by the
 * caller).  The data-gradient convs run on esr_conv3x3_fwd_x3 (linear: S passes through) with o->lrelu = 3, the
 * LeakyReLU backward through the saved split activation r2 (block.py:10-23, 233-235). */
int esr_grad_amax(const float *x, int32_t cp, int32_t coff, int32_t C, int32_t B, int32_t H, int32_t W,
                  uint32_t *amax, esr_stream_t stream);
/* out = a·x1 + b·x2 (x2 may be NULL) on C-channel slices (C % 8 == 0); each of out / x1 / x2 is fp32 or (flag 1)
 * split-f16 holding values × S(amax): split operands are read as (hi + lo) / S, a split output is written as v·S
 * (*overflow |= 1 if |v·S| >= 65504).  Channel pitches / offsets % 8 == 0. */
int esr_axpby_gs(void *out, int32_t o_cp, int32_t o_coff, int32_t o_split, float a, const void *x1, int32_t x1_cp,
                 int32_t x1_coff, int32_t x1_split, float b, const void *x2, int32_t x2_cp, int32_t x2_coff,
                 int32_t x2_split, int32_t C, int32_t B, int32_t H, int32_t W, const uint32_t *amax,
                 int32_t *overflow, esr_stream_t stream);
/* esr_axpby_gs with an fp32 output that also ORs max |out| into *out_amax (esr_grad_amax of the result, fused: the
 * x3 backward's trunk gradient at an RRDB's input is the next RRDB's gradient-scale source). */
int esr_axpby_gs_amax(float *out, int32_t o_cp, int32_t o_coff, float a, const void *x1, int32_t x1_cp, int32_t x1_coff,
                      int32_t x1_split, float b, const void *x2, int32_t x2_cp, int32_t x2_coff, int32_t x2_split,
                      int32_t C, int32_t B, int32_t H, int32_t W, const uint32_t *amax, uint32_t *out_amax,
                      esr_stream_t stream);
/* esr_wgrad_reduce / _gs with two scales: out[i] = (i < n_w ? scale_w : scale_b) [/ S(amax) if amax] · Σ_s
 * partial[s·n + i] — a conv's weights (first n_w entries) read activations of the x3 forward stored × its activation
 * scale A (scale_w carries 1/A), its bias gradient (the rest) does not. */
int esr_wgrad_reduce2(const float *partial, int32_t splits, int64_t n, int64_t n_w, float scale_w, float scale_b,
                      const uint32_t *amax, float *out, esr_stream_t stream);
/* out[i] = scale / S(amax) · Σ_s partial[s·n + i]: the weight gradient of a conv whose output gradient was scaled. */
int esr_wgrad_reduce_gs(const float *partial, int32_t splits, int64_t n, float scale, const uint32_t *amax, float *out,
                        esr_stream_t stream);
/* LeakyReLU(0.2) backward from the saved output y: d *= (y > 0 ? 1 : 0.2) on a C-channel slice. */
int esr_lrelu_bwd(float *d, int32_t d_cp, int32_t d_coff, const float *y, int32_t y_cp, int32_t y_coff, int32_t C,
                  int32_t B, int32_t H, int32_t W, esr_stream_t stream);
/* The same with y in the split-f16 layout (the x3 forward's activations; y_cp % 8 == 0). */
int esr_lrelu_bwd_split(float *d, int32_t d_cp, int32_t d_coff, const void *y, int32_t y_cp, int32_t y_coff, int32_t C,
                        int32_t B, int32_t H, int32_t W, esr_stream_t stream);
/* out = a·x1 + b·x2 (x2 may be NULL) on C-channel slices of padded NHWC buffers (in place allowed, pointwise). */
int esr_axpby(float *out, int32_t o_cp, int32_t o_coff, float a, const float *x1, int32_t x1_cp, int32_t x1_coff,
              float b, const float *x2, int32_t x2_cp, int32_t x2_coff, int32_t C, int32_t B, int32_t H, int32_t W,
              esr_stream_t stream);
/* Adjoint of nearest ×2 upsampling: out (H×W grid) = Σ over each 2×2 block of src (2H×2W grid). */
int esr_sum2x2(float *out, int32_t o_cp, int32_t o_coff, const float *src, int32_t s_cp, int32_t s_coff, int32_t C,
               int32_t B, int32_t H, int32_t W, esr_stream_t stream);
/* NCHW [B][C][H][W] <-> padded NHWC channel slice (to_nchw = 0: src -> dst; 1: dst -> src). */
int esr_nchw_to_padded(const float *src, int32_t C, int32_t B, int32_t H, int32_t W, float *dst, int32_t d_cp,
                       int32_t d_coff, int32_t to_nchw, esr_stream_t stream);
/* Exact adjoint of a replicate-padded strided depthwise stencil F(x)[o] = Σ_u w[u] x[clamp(s·o + c + u - K/2)]
 * (2-D, same s/c per dimension; x is Ly×Lx, g = F's output shape Oy×Ox, `planes` = B·C images):
 *   out[i][j] (+)= alpha · F^T(g)[os·i + oc][os·j + oc]
 * Used with (s, c, os, oc) = (1, 0, sf, ph) for Upscale_OP (adjoint sampled on the stuffed phase), (1, 0, 1, 0) for
 * Conv_LR_with_Inv_hTh_OP and (sf, ph, 1, 0) for DownscaleOP (CEMnet.py:149-162).
 * flags: bit 0 = accumulate into out (+=); bit 1 = the generic per-tap range search everywhere (default: outputs whose
 * taps see no replicate clamp visit only the contributing taps, in the generic loop's order — bitwise equal). */
int esr_cem_adjoint(const float *g, int32_t planes, int32_t Oy, int32_t Ox, const float *w, int32_t K, int32_t s,
                    int32_t c, int32_t Ly, int32_t Lx, int32_t os, int32_t oc, float alpha, int32_t flags,
                    float *out, esr_stream_t stream);

/* Input gradient of the generator (Z optimisation, Z_optimization.py:574-630): out [B][C][Hp-2M][Wp-2M] (NCHW) =
 *   RepPad_M^T( d_hr  +  d_pl  +  Bilinear↓sf^T(d_lr) )
 * where d_hr is a C-channel slice of a padded NHWC buffer at Hp×Wp, d_pl a planar [B][C][Hp][Wp] array and d_lr a
 * slice of a padded NHWC buffer at (Hp/sf)×(Wp/sf) (bilinear, align_corners=False; sf = 4: each LR pixel is the mean
 * of the central 2×2 of its 4×4 block, sf = 2: of its 2×2 block, architecture.py:153-157); any of the three may be
 * NULL.  RepPad_M is the
 * ReplicationPad2d(M) of CEM's eval-mode pre-pad (CEMnet.py:170-181; M = 0 for train mode). */
int esr_input_adjoint(const float *d_hr, int32_t hr_cp, int32_t hr_coff, const float *d_lr, int32_t lr_cp,
                      int32_t lr_coff, int32_t sf, const float *d_pl, int32_t C, int32_t B, int32_t Hp, int32_t Wp,
                      int32_t M, float *out, esr_stream_t stream);

/* ---- discriminator convolutions (esr_dconv.hip) -----------------------------------------------------------------
 * Discriminator_VGG_128_ (architecture.py:222-284): the conv_block convolutions (block.py:129-156; k = 3/4/8/1,
 * stride 1/2) of the D step and of the WGAN-GP double backward (SRRaGAN_model.py:360-433, loss.py:244-263), on
 * channels-last (NHWC, no halo) tensors.
 *
 * `prec` (every esr_dconv_* entry point, per call): 0 = exact fp32 MFMA (v_mfma_f32_32x32x2_f32); 1 = x3: both operands
 * split into f16 hi/lo at staging after a power-of-two scaling per K step (one tap × 32 channels, or per staged
 * 32-channel window in the halo kernels) chosen from the workgroup's max |a| and max |b|, products hi·hi + hi·lo +
 * lo·hi on f16 MFMA, the fp32 accumulators rescaled exactly when the step's scale changes (esr_dconv_wgrad likewise:
 * per 64-pixel K step); 128 output channels per workgroup where n_pad % 128 == 0 and the grid keeps >= 512 workgroups;
 * 2 = x3 with 64-channel N tiles only (identical results); 3 = x6: three f16 pieces hi, lo, lo2 per operand value and
 * the six products hi·hi, hi·lo, lo·hi, lo·lo, hi·lo2, lo2·hi — every dropped term below 2^-33 of the step's scale,
 * i.e. an fp32 FMA chain's accuracy.
 * Kernels (a function of the geometry): the halo-tile implicit GEMMs (each source pixel of a 32-channel chunk staged in
 * LDS once for all taps) for stride-1 launches with one tap or >= 9 taps (and the space-to-depth forms) whose width the
 * tiles cover with <= 30 % waste and whose halo fits in LDS; the per-tap gather kernels otherwise.
 *
 * esr_dconv_fwd: gather-GEMM
 *   out[b, omy*Y+oay, omx*X+oax, n] = bias[n] + sum_t sum_{c<kc} src[b, smy*Y+offy[t], smx*X+offx[t], c] * W[t][c][n]
 * for Y < MH, X < MW, n < n_out; source pixels outside [0,Hs)x[0,Ws) read as zero (the conv's zero padding).
 *   forward conv (k, s, pad):  MH x MW = output grid, omy = omx = 1, oay = oax = 0, smy = smx = s, offy = ky - pad
 *   data gradient:             one call per input phase class (cy, cx) of the stride: src = dL/dout, W[t] = w[:, :, ky,
 *                              kx] (K = Cout, N = Cin) for the taps with (cy + pad - ky) % s == 0, offy = (cy+pad-ky)/s,
 *                              smy = 1, omy = s, oay = cy (pixels of other classes are not written)
 * w_packed: [T][nck][n_pad][32] fp32 (nck = ceil(kc/32), n_pad = 64*ceil(n_out/64)); channel k of chunk j is 32j + k,
 * zero beyond kc / n_out.  bias may be NULL.  T <= ESR_DCONV_MAX_TAPS. */
#define ESR_DCONV_MAX_TAPS 64
int esr_dconv_fwd(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t kc,
                  const float *w_packed, int32_t nck, int32_t n_pad, const float *bias, float *out, int32_t Ho,
                  int32_t Wo, int32_t out_pitch, int32_t n_out, int32_t MH, int32_t MW, int32_t omy, int32_t oay,
                  int32_t omx, int32_t oax, int32_t smy, int32_t smx, int32_t T, const int32_t *offy,
                  const int32_t *offx, int32_t prec, esr_stream_t stream);
/* esr_dconv_fwd with split-K over ksplit workgroup slices of the K steps (x3) or of the 32-channel chunks (fp32
 * halo kernel) — for the small-M,
 * long-K launches — the 8×8 pseudo-FC layer — that would fill few CUs): partial = caller buffer of
 * ksplit·MH·MW·B·n_pad floats; a second kernel sums the slices in order (deterministic) and applies bias and the
 * output map.  ksplit = 1 is esr_dconv_fwd. */
int esr_dconv_fwd_sk(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t kc,
                     const float *w_packed, int32_t nck, int32_t n_pad, const float *bias, float *out, int32_t Ho,
                     int32_t Wo, int32_t out_pitch, int32_t n, int32_t MH, int32_t MW, int32_t omy, int32_t oay,
                     int32_t omx, int32_t oax, int32_t smy, int32_t smx, int32_t T, const int32_t *offy,
                     const int32_t *offx, int32_t ksplit, float *partial, int32_t prec, esr_stream_t stream);
/* The ksplit esr_dconv_fwd_sk should get for this launch geometry at precision `prec` (1 = no split); the caller
 * allocates `partial` accordingly.  Exact fp32: the halo-tile kernel splits the 32-channel chunks where its grid has
 * < 512 workgroups (the 8×8 pseudo-FC layer); x3: ~512 workgroups, >= 8 K steps per slice. */
int esr_dconv_fwd_splits(int32_t B, int32_t MH, int32_t MW, int32_t n_out, int32_t kc, int32_t smy, int32_t smx,
                         int32_t T, const int32_t *offy, const int32_t *offx, int32_t prec);
/* esr_dconv_fwd_sk over a space-to-depth source and/or into a depth-to-space output: a k×k stride-2 conv (k even) as
 * a (k/2)×(k/2)-tap stride-1 one with 4× the channels, the form the halo-tile kernel stages once per source pixel.
 *   Virtual channel order: v(py, px, c) = (c / G)·4G + (2·py + px)·G + c % G with G = 32 where the real channel
 *   count is a multiple of 32 (a 32-channel K chunk is then 128 contiguous bytes of one real pixel), else G = it.
 *   s2d_c > 0 (forward): src is the REAL [B][Hs][Ws][src_pitch] input with s2d_c channels (a multiple of 4) and
 *     kc = 4·s2d_c; virtual channel v(py, px, c) of virtual pixel (sy, sx) = src[b, 2·sy + py - s2d_pad,
 *     2·sx + px - s2d_pad, c] (zero outside), so with W[(a, b)][v(py, px, c)][n] = w[n][c][2a + py][2b + px],
 *     offy = a, offx = b, smy = smx = 1 this is conv2d(src, w, stride 2, padding s2d_pad).
 *   d2s_c > 0 (data gradient): n_out = 4·d2s_c, out is the REAL [B][Ho][Wo][out_pitch] input gradient; virtual
 *     channel v(py, px, c) of grid point (Y, X) goes to out[b, 2·Y + py - d2s_pad, 2·X + px - d2s_pad, c]
 *     (dropped outside); omy = omx = 1, oay = oax = 0, no bias.  With src = dL/dy, offy = -a, offx = -b and
 *     W[(a, b)][co][v(py, px, c)] = w[co][c][2a + py][2b + px] over MH × MW = ((H-1+pad)/2 + 1) × ((W-1+pad)/2 + 1)
 *     this is the transposed conv in one launch (replaces the per-phase-class calls of esr_dconv_fwd).
 * w_split / w_exp (both NULL, or both given; prec 1 / 2): the weights pre-split for the x3 halo-tile kernel — the
 *   values of w_packed times 2^E (E = *w_exp, one power of two per tensor, |w|·2^E < 2^15) as f16 hi and lo =
 *   f16(v - hi): per (tap t, chunk j, output channel n) one 128-byte row of eight 16-byte slots, logical slot l =
 *   piece·4 + k (piece 0 hi, 1 lo; k-th group of 8 channels of the chunk) stored at position l ^ ((n >> 1) & 7),
 *   rows [T][nck][n_pad].  Halo-tile launches then LDS-DMA them (no per-step max, split or register staging);
 *   other launches use w_packed.
 * Replaces: the D's 4×4 stride-2 conv_block convs (architecture.py:232-250, block.py:129-156) and their gradients. */
int esr_dconv_fwd_sd(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t kc,
                     const float *w_packed, int32_t nck, int32_t n_pad, const float *bias, float *out, int32_t Ho,
                     int32_t Wo, int32_t out_pitch, int32_t n, int32_t MH, int32_t MW, int32_t omy, int32_t oay,
                     int32_t omx, int32_t oax, int32_t smy, int32_t smx, int32_t T, const int32_t *offy,
                     const int32_t *offx, int32_t ksplit, float *partial, int32_t s2d_c, int32_t s2d_pad,
                     int32_t d2s_c, int32_t d2s_pad, int32_t prec, const void *w_split, const int32_t *w_exp,
                     esr_stream_t stream);
/* The w_split / w_exp form of a packed weight tensor (rows = T·nck·n_pad rows of 32 floats): two launches (a partial
 * max over ESR_DCONV_PRESPLIT_SCRATCH floats of scratch, then the split), no host synchronisation. */
#define ESR_DCONV_PRESPLIT_SCRATCH 512
int esr_dconv_presplit(const float *w_packed, int64_t rows, int32_t n_pad, float *scratch, void *w_split,
                       int32_t *w_exp, esr_stream_t stream);

/* The discriminator's first conv (3 input channels, 3×3, stride 1: architecture.py:229) runs as a 1×1 conv over its
 * taps gathered into one 32-wide K step.  esr_dconv_im2col: out [B][Ho][Wo][32] (Ho = H + 2p - k + 1) with
 * out[..][t·C + c] = x[b][y + ky - p][x + kx - p][c] (zero outside the image), t = ky·k + kx, zero-filled past k²·C
 * (k²·C <= 32; out 16-B aligned).  esr_dconv_col2im: its adjoint, gx [B][H][W][C] = Σ_t (in tap order, from 0)
 * gc[b][y - ky + p][x - kx + p][t·C + c] over the outputs in range (C <= 8).  x, gx NHWC [B][H][W][C]. */
int esr_dconv_im2col(const float *x, int32_t B, int32_t H, int32_t W, int32_t C, int32_t k, int32_t p, float *out,
                     esr_stream_t stream);
int esr_dconv_col2im(const float *gc, int32_t B, int32_t H, int32_t W, int32_t C, int32_t k, int32_t p, float *gx,
                     esr_stream_t stream);
/* The discriminator's first conv block fused (architecture.py:231 -> block.py:129-156: Conv2d(3, 64, 3, stride 1,
 * padding 1) + LeakyReLU(slope), no norm), exact fp32 on the VALU (csrc/esr_dfirst.hip).  x [B][H][W][3] NHWC,
 * w [64][3][3][3] (torch layout), bias [64] or NULL, y / mask [B][H][W][64] (16-B aligned).
 * esr_dfirst_fwd: y = conv(x, w) + bias, then per flags: ESR_DFIRST_ACC adds y's previous contents, ESR_DFIRST_LRELU
 * applies LeakyReLU(slope), ESR_DFIRST_MASK multiplies by lrelu'(mask) (mask: the layer's saved output, its sign the
 * LeakyReLU mask; the double backward's path).
 * esr_dfirst_bwd (x may be NULL when partial is): with g' = gy · lrelu'(mask) (mask NULL: g' = gy): gx (if non-NULL) = the input gradient
 * Σ w[co][ci][ky][kx] g'[y - ky + 1][x - kx + 1][co] (written, not added); partial (if non-NULL) = per block b of
 * esr_dfirst_bwd_blocks(B, H, W) blocks, ESR_DFIRST_NW floats at b·ESR_DFIRST_NW: the weight gradient
 * Σ x[y + ky - 1][x + kx - 1][ci] g'[y][x][co] at co·27 + ci·9 + ky·3 + kx, then the bias gradient Σ g'[co] at
 * 1728 + co, over the block's pixels — sum the blocks with esr_wgrad_reduce(partial, blocks, ESR_DFIRST_NW, 1, out). */
#define ESR_DFIRST_COUT 64
#define ESR_DFIRST_NW (64 * 27 + 64)
#define ESR_DFIRST_LRELU 1
#define ESR_DFIRST_MASK 2
#define ESR_DFIRST_ACC 4
int esr_dfirst_fwd(const float *x, int32_t B, int32_t H, int32_t W, const float *w, const float *bias, float slope,
                   int32_t flags, const float *mask, float *y, esr_stream_t stream);
/* esr_dfirst_fwd on the padded NHWC records of the generator's backward (halo 1, zero): x [B][H+2][W+2][x_cp] (3
 * channels at 0), y [B][H+2][W+2][y_cp] at channel y_coff, interior written (flags: LRELU / ACC).  HR_conv1's data
 * gradient (architecture.py:141) is this 3 -> 64 3×3 conv with its weights flipped and transposed. */
int esr_dfirst_fwd_padded(const float *x, int32_t x_cp, int32_t B, int32_t H, int32_t W, const float *w,
                          const float *bias, float slope, int32_t flags, float *y, int32_t y_cp, int32_t y_coff,
                          esr_stream_t stream);
int esr_dfirst_bwd_blocks(int32_t B, int32_t H, int32_t W);
int esr_dfirst_bwd(const float *x, const float *gy, const float *mask, float slope, int32_t B, int32_t H, int32_t W,
                   const float *w, float *gx, float *partial, esr_stream_t stream);
/* 1 if an esr_dconv_fwd(_sd) launch of this geometry runs on the halo-tile kernel (sd != 0: an esr_dconv_fwd_sd
 * launch), 0 if on the per-tap gather kernel.  The host takes the space-to-depth forward only where it is halo-tiled
 * (on the gather kernel it is no faster than the direct stride-2 gather: profiles/r3_dconv_s2d_ab.txt). */
int esr_dconv_uses_halo(int32_t smy, int32_t smx, int32_t T, int32_t MW, int32_t sd, int32_t prec);
/* esr_dconv_fwd_splits for an esr_dconv_fwd_sd launch (sd != 0: space-to-depth source or depth-to-space output). */
int esr_dconv_fwd_splits_sd(int32_t B, int32_t MH, int32_t MW, int32_t n_out, int32_t kc, int32_t smy, int32_t smx,
                            int32_t T, const int32_t *offy, const int32_t *offx, int32_t sd, int32_t prec);
/* esr_dconv_wgrad: weight gradient of the forward conv above (src = its input, dy = dL/dout on the MH x MW grid):
 *   partial[s][t][ci][co] = sum over the pixels of split s of src[b, smy*Y+offy[t], smx*X+offx[t], ci] * dy[b, Y, X, co]
 * partial: [splits][T][cin_pad][cout_pad], cin_pad = 64*ceil(cin/64), cout_pad = 64*ceil(cout/64); reduce the splits
 * with esr_wgrad_reduce (fixed order, deterministic). */
/* The `splits` esr_dconv_wgrad should get for this geometry at precision `prec` (the caller sizes `partial` with it).
 * Returns ESR_EINVAL on bad arguments. */
int esr_dconv_wgrad_splits(int32_t B, int32_t MH, int32_t MW, int32_t cin, int32_t cout, int32_t smy, int32_t smx,
                           int32_t T, const int32_t *offy, const int32_t *offx, int32_t prec);
int esr_dconv_wgrad(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t cin,
                    const float *dy, int32_t MH, int32_t MW, int32_t dy_pitch, int32_t cout, int32_t smy, int32_t smx,
                    int32_t T, const int32_t *offy, const int32_t *offx, int32_t splits, float *partial,
                    int32_t prec, esr_stream_t stream);

/* ---- op lists (host-side executor, esr_plan.hip) -----------------------------------------------------------------
 * A generator (+CEM) forward is a fixed sequence of the launches above (≈360 for RRDB-23).  The host layer records it
 * once per (workspace, weights, shape) as an array of esr_op and replays it with one esr_run_ops call, patching only
 * the input / output pointers between calls; esr_run_ops optionally brackets every op with HIP events (esr_timer_*)
 * for per-kernel timing inside the benchmark's timed region.  Argument order per kind (p = pointers, i = int32s):
 *   CONV3X3     p: in, w, bias           i: B, H, W, in_cp, cin, cout              + o
 *   CONV3X3_X3  p: in, w, bias, overflow i: B, H, W, in_cp, cin, cout   f0: w_scale + o
 *   UPCONV      p: in, w, bias           i: B, H, W, in_cp, cin, cout, py, px      + o
 *   UPCONV_X3   p: in, w, bias, overflow i: B, H, W, in_cp, cin, cout, py, px  f0 + o
 *   PREP        p: x, lr_nchw, first, zlr[4], zhr[2]
 *               i: B, nz, h, w, sf, m, first_cp, first_lr_off, zlr_cp[4], n_zlr, zhr_cp[2], n_zhr, split
 *   CEM_DOWN    p: gen, lr, r, w_down    i: B, H, W, sf, ph, kd, negate
 *   CEM_INV     p: r, q, w_inv           i: B, H, W, ki
 *   CEM_UP_ADD  p: q, gen, out, w_up     i: B, H, W, sf, ph, kd, M
 *   HR_CONVS_X3 p: in, w0, bias0, w1, y, overflow   i: B, H, W, in_cp, zc   f0: w0_scale
 *   HR1_SUM     p: y, bias1, out         i: B, H, W                  f0: scale_inv               */
enum esr_op_kind {
    ESR_OP_CONV3X3 = 1,
    ESR_OP_CONV3X3_X3 = 2,
    ESR_OP_UPCONV = 3,
    ESR_OP_UPCONV_X3 = 4,
    ESR_OP_PREP = 5,
    ESR_OP_CEM_DOWN = 6,
    ESR_OP_CEM_INV = 7,
    ESR_OP_CEM_UP_ADD = 8,
    ESR_OP_HR_CONVS_X3 = 9,
    ESR_OP_HR1_SUM = 10,
};
typedef struct esr_op {
    int32_t kind;
    int32_t tag; /* caller's label (profiling) */
    const void *p[10];
    int32_t i[20];
    float f[2];
    esr_conv_out o;
} esr_op;
typedef void *esr_timer_t;
esr_timer_t esr_timer_create(int32_t n_ops);            /* n_ops + 1 HIP events; NULL on failure */
int esr_timer_elapsed(esr_timer_t timer, float *ms);    /* waits; ms[k] = duration of op k of the last run */
void esr_timer_destroy(esr_timer_t timer);
/* Event k (0..n_ops) of `timer` recorded on `stream` now (a reference mark: a timer of one op, event 0). */
int esr_timer_record(esr_timer_t timer, int32_t k, esr_stream_t stream);
/* Waits; t_ms[k] (k = 0..n_ops) = time of event k of the last run relative to event 0 of `ref`: the absolute launch
 * intervals [t_ms[k], t_ms[k+1]] of op lists run on several streams at once (bench.py's roofline over their union). */
int esr_timer_stamps(esr_timer_t timer, esr_timer_t ref, float *t_ms);
int esr_run_ops(const esr_op *ops, int32_t n, esr_timer_t timer, esr_stream_t stream);
int esr_op_size(void);                                  /* sizeof(esr_op), checked by the binding */

/* ---- discriminator BatchNorm2d (training) + LeakyReLU (esr_bn.hip) ------------------------------------------------
 * conv_block(CNA)'s norm + act (block.py:129-156) fused on channels-last activations x [P][C] (P = B·H·W):
 *   μ, v = batch mean / biased variance per channel, r = 1/sqrt(v + eps), y = lrelu_slope(γ·(x − μ)·r + β).
 * esr_bn_lrelu_fwd writes y and the per-channel mu, rs (= r) and var, and, when running_mean / running_var are set,
 * updates them as nn.BatchNorm2d does (momentum in [0, 1]: r = r·(1 − m) + m·μ, rv = rv·(1 − m) + m·P/(P−1)·v) and adds
 * 1 to *num_batches_tracked (int64; may be NULL).
 * esr_bn_lrelu_bwd: gx = ∂L/∂x for upstream gy, and sums2 = [Σ gz ; Σ gz·x̂] (= dβ ; dγ), gz = gy·lrelu'.
 * esr_bn_lrelu_bwd2: the backward of (x, γ, gy) -> (gx, dγ, dβ) (the WGAN-GP double backward, loss.py:244-263) for
 * upstream u = ∂/∂gx, ggg = ∂/∂dγ, ggb = ∂/∂dβ (each may be NULL = 0): g_x, g_gy and g_gamma (formulas in
 * esr_bn.hip's header).  ws = scratch of esr_bn_workspace_floats(P, C) floats.  Deterministic (fixed-order sums). */
int64_t esr_bn_workspace_floats(int64_t P, int32_t C);
/* out[c] = Σ_p x[p][c] over a [P][C] float tensor, float64 partial sums in fixed order (bn_colsum + bn_finish); ws as
 * above.  The discriminator convs' bias gradients (Σ of the output gradient over batch and pixels): PyTorch's
 * reduction of an NHWC [B, H, W, C] tensor over (0, 1, 2) ran at ~0.2 TB/s. */
int esr_colsum(const float *x, int64_t P, int32_t C, float *out, float *ws, esr_stream_t stream);
int esr_bn_lrelu_fwd(const float *x, int64_t P, int32_t C, const float *gamma, const float *beta, float eps,
                     float slope, float *y, float *mu, float *rs, float *var, float *ws, float *running_mean,
                     float *running_var, int64_t *num_batches_tracked, float momentum, esr_stream_t stream);
int esr_bn_lrelu_bwd(const float *x, const float *gy, int64_t P, int32_t C, const float *gamma, const float *beta,
                     const float *mu, const float *rs, float slope, float *gx, float *sums2, float *ws,
                     esr_stream_t stream);
int esr_bn_lrelu_bwd2(const float *x, const float *gy, const float *u, const float *ggg, const float *ggb, int64_t P,
                      int32_t C, const float *gamma, const float *beta, const float *mu, const float *rs, float slope,
                      const float *sums2, float *g_x, float *g_gy, float *g_gamma, float *ws, esr_stream_t stream);

/* Library / ABI version (bumped on any signature change). */
int esr_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ESR_AMD_H */
