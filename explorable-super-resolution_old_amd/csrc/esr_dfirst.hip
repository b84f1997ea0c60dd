// esr_dfirst.hip — the discriminator's first conv block (architecture.py:231: conv_block(in_nc = 3, base_nf = 64,
// kernel_size = 3, norm None, act LeakyReLU 0.2) -> block.py:129-156: Conv2d(3, 64, 3, padding 1) + LeakyReLU), fused,
// on the VALU in exact fp32.
//
// With 3 input channels the conv is 27 MACs per output: there is no K dimension to feed the matrix cores, and the
// layer's cost is moving its 64-channel output (the largest activation of the discriminator: 16·304²·64 floats =
// 378 MB at config 3).  The general path (im2col to 32 columns + a 1×1 split-f16 MFMA conv + a separate LeakyReLU
// pass, and for the backward a LeakyReLU-backward pass, a 1×1 data-gradient conv, col2im, the wgrad conv and a bias
// sum) moved that tensor 4-6 times per pass.  Here:
//   forward   one pass: 27 inputs per pixel from L1, 64 outputs per thread, weights uniform per block (scalar
//             loads), bias + LeakyReLU in the store, the block's 256 × 64 outputs restaged through LDS one
//             32-channel half at a time so that a store instruction writes whole 128-B half-records;
//   backward  one pass over (gy, y): g' = gy · lrelu'(y) staged per 16-channel chunk for a tile + 1-pixel halo (the
//             weights transposed in LDS: 3 broadcast reads per tap and 4 channels; as scalar loads, scattered, the
//             pass took 1.39 ms instead of 0.51 at config 3), the
//             input gradient (27 taps × 16 channels per chunk per pixel) and the per-block weight / bias partial sums
//             from the same LDS tile; a deterministic second pass (esr_wgrad_reduce) adds the block partials in order.
// Results are exact fp32 (one rounding per FMA), at least as accurate as every `prec` of the general path.
#include <hip/hip_runtime.h>
#include "esr_amd.h"

namespace {

inline int launched() { return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH; }

constexpr int CO = ESR_DFIRST_COUT;  // 64 output channels
constexpr int KT = 27;               // 3 input channels × 3 × 3 taps, torch order ci·9 + ky·3 + kx
constexpr int NW = ESR_DFIRST_NW;    // weight-gradient entries per block partial: 64 · 27 weights + 64 biases

__device__ __forceinline__ float lrelu_mask(float m, float slope) { return m > 0.f ? 1.f : slope; }

// ---- forward ---------------------------------------------------------------------------------------------------
// Thread = one output pixel (flat index over [B][H][W]), 64 accumulators; block = 256 consecutive pixels.
// flags: ESR_DFIRST_LRELU: LeakyReLU(slope) of the sum; ESR_DFIRST_MASK: the sum times lrelu'(m) (m = the forward's
// saved output: the double backward's data-gradient path); ESR_DFIRST_ACC: the previous contents of y are added
// to the sum first (before the mask).
constexpr int F_BLK = 256, F_HALF = CO / 2, F_PITCH = F_HALF + 4;
// Layouts: pad = 0: x [B][H][W][x_cp], y / m [B][H][W][64] (y_cp = 64, y_coff = 0); pad = 1: the padded NHWC records
// of the generator's backward, x [B][H+2][W+2][x_cp] (3 channels at 0), y [B][H+2][W+2][y_cp] at channel y_coff (no
// mask), interior pixels only.
__global__ __launch_bounds__(F_BLK) void dfirst_fwd_kernel(const float *__restrict__ x, long long P, int H, int W,
                                                           const float *__restrict__ w, const float *__restrict__ bias,
                                                           float slope, int flags, const float *__restrict__ m,
                                                           float *__restrict__ y, int x_cp, int pad, int y_cp,
                                                           int y_coff) {
    // the outputs restaged through LDS one 32-channel half at a time (36 KB: four blocks per CU)
    __shared__ __attribute__((aligned(16))) float s[F_BLK * F_PITCH];
    const long long p0 = (long long)blockIdx.x * F_BLK;
    const long long p = p0 + threadIdx.x;
    float xin[KT];
    if (p < P) {
        const int xx = (int)(p % W);
        const long long r = p / W;
        const int yy = (int)(r % H);
        const long long b = r / H;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int Y = yy + ky - 1, X = xx + kx - 1;
                const bool in = Y >= 0 && Y < H && X >= 0 && X < W;
                const float *src = x + (pad ? ((b * (H + 2) + Y + 1) * (W + 2) + X + 1) : ((b * H + Y) * W + X)) * x_cp;
#pragma unroll
                for (int ci = 0; ci < 3; ++ci) xin[ci * 9 + ky * 3 + kx] = in ? src[ci] : 0.f;
            }
    } else {
#pragma unroll
        for (int k = 0; k < KT; ++k) xin[k] = 0.f;
    }
    float *row = s + threadIdx.x * F_PITCH;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h) __syncthreads();  // the first half's stores have read the stage
#pragma unroll
        for (int c4 = 0; c4 < F_HALF / 4; ++c4) {
            float a[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                // uniform over the block: scalar loads of 27 consecutive floats (faster here than LDS broadcasts:
                // 169 vs 219 us at config 3)
                const int co = F_HALF * h + 4 * c4 + j;
                const float *wc = w + co * KT;
                float v = 0.f;
#pragma unroll
                for (int k = 0; k < KT; ++k) v = fmaf(wc[k], xin[k], v);
                a[j] = bias ? v + bias[co] : v;
            }
            *reinterpret_cast<float4 *>(row + 4 * c4) = make_float4(a[0], a[1], a[2], a[3]);
        }
        __syncthreads();
        // store: 256 pixels × 8 float4 of this half, consecutive threads -> consecutive float4 (128 B per pixel)
#pragma unroll 4
        for (int k = 0; k < F_HALF / 4; ++k) {
            const int idx = threadIdx.x + F_BLK * k, px = idx >> 3, c = 4 * (idx & 7);
            const long long q = p0 + px;
            if (q >= P) continue;
            float4 v = *reinterpret_cast<const float4 *>(s + px * F_PITCH + c);
            long long rec = q;  // output record of pixel q
            if (pad) {
                const long long xx = q % W, r = q / W, yy = r % H, bb = r / H;
                rec = (bb * (H + 2) + yy + 1) * (W + 2) + xx + 1;
            }
            float *dst = y + rec * y_cp + y_coff + F_HALF * h + c;
            if (flags & ESR_DFIRST_ACC) {
                const float4 o = *reinterpret_cast<const float4 *>(dst);
                v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
            }
            if (flags & ESR_DFIRST_LRELU) {
                v.x = v.x > 0.f ? v.x : v.x * slope; v.y = v.y > 0.f ? v.y : v.y * slope;
                v.z = v.z > 0.f ? v.z : v.z * slope; v.w = v.w > 0.f ? v.w : v.w * slope;
            }
            if (flags & ESR_DFIRST_MASK) {
                const float4 mm = *reinterpret_cast<const float4 *>(m + q * CO + F_HALF * h + c);
                v.x *= lrelu_mask(mm.x, slope); v.y *= lrelu_mask(mm.y, slope);
                v.z *= lrelu_mask(mm.z, slope); v.w *= lrelu_mask(mm.w, slope);
            }
            *reinterpret_cast<float4 *>(dst) = v;
        }
    }
}

// ---- backward --------------------------------------------------------------------------------------------------
// Block = 256 threads (4 waves) over 8 × 32-pixel output tiles (tile t = blockIdx.x + k·gridDim.x).  Per tile: the
// input on the tile + halo (10 × 34 pixels × 3) and, per 32-channel chunk, g' = gy · lrelu'(m) on the tile + halo in
// LDS.
//   input gradient (VALU, thread = tile pixel): gx[r][ci] = Σ_{ky,kx,co} w[co][ci][ky][kx] · g'[r − (ky−1, kx−1)][co]
//     with the weights transposed in LDS (3 broadcast reads per tap and 4 channels; as scattered scalar loads the
//     pass took 1.39 instead of 0.51 ms at config 3);
//   weight / bias gradient (fp32 MFMA v_mfma_f32_16x16x4f32, wave w = tile rows 2w, 2w + 1): per chunk
//     D[co][n] += Σ_p g'[p][co] · X[p][n] over the wave's 64 pixels, 4 per K step, where X[p][n] = x[p + tap(n) − 1]
//     [ci(n)] for the 27 (ci, tap) entries n = ci·9 + tap, X[p][27] = 1 (the bias gradient: column 27 of D) and 0 for
//     n = 28..31 (two 16-channel M tiles per chunk).  At the end of each chunk's pass the 4 waves' sums are added in
//     wave order and the block writes that chunk's part of its NW partial sums.
constexpr int B_TY = 8, B_TX = 32, B_HY = B_TY + 2, B_HX = B_TX + 2, B_HP = B_HY * B_HX;  // 340 halo pixels
// g' chunk channels (32: a chunk's 128 B of a pixel are one whole cache line — with 16-channel chunks every chunk pass
// fetched whole lines for half of them, twice the HBM traffic), LDS pitch (floats), 16-row MFMA M tiles per chunk
constexpr int B_CC = 32, B_GP = B_CC + 4, B_MT = B_CC / 16;
constexpr int B_RED = 4 * B_MT * 2 * 4 * 64;                   // one chunk's accumulators of the 4 waves (floats)
constexpr int B_SG = B_HP * B_GP > B_RED ? B_HP * B_GP : B_RED;
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void dfirst_bwd_kernel(const float *__restrict__ x, const float *__restrict__ gy,
                                                         const float *__restrict__ m, float slope, int B, int H, int W,
                                                         const float *__restrict__ w, float *__restrict__ gx,
                                                         float *__restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float sg[B_SG];
    __shared__ float sx[B_HP * 3];
    __shared__ __attribute__((aligned(16))) float wt[9 * CO * 3];  // w[co][ci][tap] at (tap·64 + co)·3 + ci
    const int t = threadIdx.x;
    for (int i = t; gx && i < CO * KT; i += 256) {
        const int co = i / KT, k = i - KT * co, ci = k / 9, tap = k - 9 * ci;
        wt[(tap * CO + co) * 3 + ci] = w[i];
    }
    const int tiles_x = (W + B_TX - 1) / B_TX, tiles_y = (H + B_TY - 1) / B_TY;
    const long long ntiles = (long long)B * tiles_y * tiles_x;
    // weight-gradient role: wave rows 2w, 2w+1; lane = (K index kq of a K step, M / N index ml)
    const int wave = t >> 6, lane = t & 63, kq = lane >> 4, ml = lane & 15;
    int xo[2];  // this lane's X column n = 16 nt + ml: offset in sx from a pixel's halo origin; -1 = 1, -2 = 0
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int n = 16 * nt + ml;
        if (n < KT) {
            const int ci = n / 9, tap = n - 9 * ci, ky = tap / 3, kx = tap - 3 * ky;
            xo[nt] = (ky * B_HX + kx) * 3 + ci;
        } else {
            xo[nt] = n == KT ? -1 : -2;
        }
    }
    const int ty = t >> 5, tx = t & 31;  // input-gradient role: this tile pixel
    float *out = partial ? partial + (long long)blockIdx.x * NW : nullptr;
    // chunk-outer (the weight-gradient accumulators of one chunk only: 8 registers, not 32); the input gradient is
    // carried across chunks through gx (chunk 0 writes, the others continue the same FMA chain from the stored value)
    for (int c = 0; c < CO / B_CC; ++c) {
        f32x4_t acc[B_MT][2];
#pragma unroll
        for (int mt = 0; mt < B_MT; ++mt) acc[mt][0] = acc[mt][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
            const int txi = (int)(tile % tiles_x);
            const long long r = tile / tiles_x;
            const int tyi = (int)(r % tiles_y);
            const long long b = r / tiles_y;
            const int y0 = tyi * B_TY, x0 = txi * B_TX;
            __syncthreads();  // the previous tile's LDS reads are done
            {  // every load of the tile's windows in flight before the first use (4 of x, 6 per g' operand per thread)
                constexpr int QP = B_CC / 4;  // float4 per pixel and chunk
                constexpr int IX = (B_HP * 3 + 255) / 256, IT = (B_HP * QP + 255) / 256;
                float xv[IX];
#pragma unroll
                for (int k = 0; k < IX; ++k) {  // (x: read by the weight gradient only; may be NULL)
                    const int i = t + 256 * k, hp = i / 3, ci = i - 3 * hp, hy = hp / B_HX, hx = hp - hy * B_HX;
                    const int Y = y0 + hy - 1, X = x0 + hx - 1;
                    xv[k] = 0.f;
                    if (partial && i < B_HP * 3 && Y >= 0 && Y < H && X >= 0 && X < W)
                        xv[k] = x[((b * H + Y) * W + X) * 3 + ci];
                }
                float4 v[IT], mm[IT];
#pragma unroll
                for (int k = 0; k < IT; ++k) {
                    const int i = t + 256 * k, hp = i / QP, q = i % QP, hy = hp / B_HX, hx = hp - hy * B_HX;
                    const int Y = y0 + hy - 1, X = x0 + hx - 1;
                    v[k] = mm[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (i < B_HP * QP && Y >= 0 && Y < H && X >= 0 && X < W) {
                        const long long o = ((b * H + Y) * W + X) * CO + B_CC * c + 4 * q;
                        v[k] = *reinterpret_cast<const float4 *>(gy + o);
                        if (m) mm[k] = *reinterpret_cast<const float4 *>(m + o);
                    }
                }
#pragma unroll
                for (int k = 0; k < IT; ++k) {
                    const int i = t + 256 * k, hp = i / QP, q = i % QP;
                    if (i >= B_HP * QP) break;
                    float4 g = v[k];
                    if (m) {
                        g.x *= lrelu_mask(mm[k].x, slope); g.y *= lrelu_mask(mm[k].y, slope);
                        g.z *= lrelu_mask(mm[k].z, slope); g.w *= lrelu_mask(mm[k].w, slope);
                    }
                    *reinterpret_cast<float4 *>(sg + hp * B_GP + 4 * q) = g;
                }
#pragma unroll
                for (int k = 0; k < IX; ++k)
                    if (t + 256 * k < B_HP * 3) sx[t + 256 * k] = xv[k];
            }
            __syncthreads();
            if (gx) {
                const int Y = y0 + ty, X = x0 + tx;
                const bool in = Y < H && X < W;
                float *d = gx + ((b * H + Y) * W + X) * 3;
                float ga[3] = {0.f, 0.f, 0.f};
                if (c && in) {
                    ga[0] = d[0];
                    ga[1] = d[1];
                    ga[2] = d[2];
                }
#pragma unroll 1
                for (int tap = 0; tap < 9; ++tap) {
                    const int ky = tap / 3, kx = tap - 3 * ky;
                    const float *g = sg + ((ty + 2 - ky) * B_HX + tx + 2 - kx) * B_GP;
#pragma unroll
                    for (int q = 0; q < B_CC / 4; ++q) {
                        const float4 g4 = *reinterpret_cast<const float4 *>(g + 4 * q);
                        const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
                        // the 4 channels' 3 input-channel weights of this tap: 12 floats, 3 broadcast reads
                        const float4 *w4 = reinterpret_cast<const float4 *>(wt + (tap * CO + B_CC * c + 4 * q) * 3);
                        const float4 wa = w4[0], wb = w4[1], wc = w4[2];
                        const float wv[12] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w, wc.x, wc.y, wc.z, wc.w};
#pragma unroll
                        for (int j2 = 0; j2 < 4; ++j2)
#pragma unroll
                            for (int ci = 0; ci < 3; ++ci) ga[ci] = fmaf(wv[3 * j2 + ci], gv[j2], ga[ci]);
                    }
                }
                if (in) {
                    d[0] = ga[0];
                    d[1] = ga[1];
                    d[2] = ga[2];
                }
            }
            if (partial) {
#pragma unroll 4
                for (int st = 0; st < 16; ++st) {
                    const int pp = 4 * st + kq, py = 2 * wave + (pp >> 5), px = pp & 31;
                    const float *xs = sx + (py * B_HX + px) * 3;
                    const float *gp = sg + ((py + 1) * B_HX + px + 1) * B_GP + ml;  // g'[pixel][16 mt + ml]
                    float bv[2];
#pragma unroll
                    for (int nt = 0; nt < 2; ++nt) bv[nt] = xo[nt] >= 0 ? xs[xo[nt]] : (xo[nt] == -1 ? 1.f : 0.f);
#pragma unroll
                    for (int mt = 0; mt < B_MT; ++mt) {
                        const float a = gp[16 * mt];
#pragma unroll
                        for (int nt = 0; nt < 2; ++nt)
                            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[nt], acc[mt][nt], 0, 0, 0);
                    }
                }
            }
        }
        if (!partial) continue;
        // D[co][n] of this chunk, lane l, register r: co = 4 (l >> 4) + r, n = 16 nt + (l & 15); waves added in order
        __syncthreads();
#pragma unroll
        for (int mt = 0; mt < B_MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) sg[(((wave * B_MT + mt) * 2 + nt) * 4 + rr) * 64 + lane] = acc[mt][nt][rr];
        __syncthreads();
        for (int e = t; e < B_CC * 28; e += 256) {
            const int co = e / 28, n = e - 28 * co, nt = n >> 4, mt = co >> 4, cl = co & 15;
            const int l = 16 * (cl >> 2) + (n & 15), rr = cl & 3;
            float v = 0.f;
            for (int wv = 0; wv < 4; ++wv) v += sg[(((wv * B_MT + mt) * 2 + nt) * 4 + rr) * 64 + l];
            if (n < KT)
                out[(B_CC * c + co) * KT + n] = v;
            else
                out[CO * KT + B_CC * c + co] = v;
        }
    }
}

}  // namespace

extern "C" int esr_dfirst_fwd(const float *x, int32_t B, int32_t H, int32_t W, const float *w, const float *bias,
                              float slope, int32_t flags, const float *mask, float *y, esr_stream_t stream) {
    if (!x || !w || !y || B <= 0 || H <= 0 || W <= 0 || (flags & ~7) || ((flags & ESR_DFIRST_MASK) && !mask))
        return ESR_EINVAL;
    if (((uintptr_t)y & 15) || (mask && ((uintptr_t)mask & 15))) return ESR_EINVAL;
    const long long P = (long long)B * H * W;
    hipLaunchKernelGGL(dfirst_fwd_kernel, dim3((unsigned)((P + F_BLK - 1) / F_BLK)), dim3(F_BLK), 0,
                       (hipStream_t)stream, x, P, H, W, w, bias, slope, flags, mask, y, 3, 0, CO, 0);
    return launched();
}

extern "C" int esr_dfirst_fwd_padded(const float *x, int32_t x_cp, int32_t B, int32_t H, int32_t W, const float *w,
                                     const float *bias, float slope, int32_t flags, float *y, int32_t y_cp,
                                     int32_t y_coff, esr_stream_t stream) {
    if (!x || !w || !y || B <= 0 || H <= 0 || W <= 0 || x_cp < 3 || (flags & ~(ESR_DFIRST_LRELU | ESR_DFIRST_ACC)) ||
        y_coff < 0 || y_coff + CO > y_cp || (y_cp | y_coff) % 4 || ((uintptr_t)y & 15))
        return ESR_EINVAL;
    const long long P = (long long)B * H * W;
    hipLaunchKernelGGL(dfirst_fwd_kernel, dim3((unsigned)((P + F_BLK - 1) / F_BLK)), dim3(F_BLK), 0,
                       (hipStream_t)stream, x, P, H, W, w, bias, slope, flags, nullptr, y, x_cp, 1, y_cp, y_coff);
    return launched();
}

extern "C" int esr_dfirst_bwd_blocks(int32_t B, int32_t H, int32_t W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    const long long ntiles = (long long)B * ((H + B_TY - 1) / B_TY) * ((W + B_TX - 1) / B_TX);
    return (int)(ntiles < 512 ? ntiles : 512);  // two blocks per CU (60 KB of LDS)
}

extern "C" int esr_dfirst_bwd(const float *x, const float *gy, const float *mask, float slope, int32_t B, int32_t H,
                              int32_t W, const float *w, float *gx, float *partial, esr_stream_t stream) {
    if (!gy || !w || B <= 0 || H <= 0 || W <= 0 || (!gx && !partial) || (partial && !x)) return ESR_EINVAL;
    if (((uintptr_t)gy & 15) || (mask && ((uintptr_t)mask & 15))) return ESR_EINVAL;
    const int g = esr_dfirst_bwd_blocks(B, H, W);
    hipLaunchKernelGGL(dfirst_bwd_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, x, gy, mask, slope, B, H, W, w,
                       gx, partial);
    return launched();
}
