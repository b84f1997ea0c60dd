// esr_dfirst.hip — the discriminator's first conv block (architecture.py:231: conv_block(in_nc = 3, base_nf = 64,
// kernel_size = 3, norm None, act LeakyReLU 0.2) -> block.py:129-156: Conv2d(3, 64, 3, padding 1) + LeakyReLU), fused,
// on the VALU in exact fp32.
//
// With 3 input channels the conv is 27 MACs per output: there is no K dimension to feed the matrix cores, and the
// layer's cost is moving its 64-channel output (the largest activation of the discriminator: 16·304²·64 floats =
// 378 MB at config 3).  The general path (im2col to 32 columns + a 1×1 split-f16 MFMA conv + a separate LeakyReLU
// pass, and for the backward a LeakyReLU-backward pass, a 1×1 data-gradient conv, col2im, the wgrad conv and a bias
// sum) moved that tensor 4-6 times per pass.  Here:
//   forward   one pass: 27 inputs per pixel from L1, 64 accumulators per thread, weights uniform per wave (scalar
//             loads), bias + LeakyReLU in the store, the block's 256 × 64 outputs restaged through LDS so that
//             every store instruction writes 1 KB contiguous;
//   backward  one pass over (gy, y): g' = gy · lrelu'(y) staged per 16-channel chunk for a tile + 1-pixel halo, the
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
constexpr int F_BLK = 256, F_PITCH = CO + 4;
__global__ __launch_bounds__(F_BLK) void dfirst_fwd_kernel(const float *__restrict__ x, long long P, int H, int W,
                                                           const float *__restrict__ w, const float *__restrict__ bias,
                                                           float slope, int flags, const float *__restrict__ m,
                                                           float *__restrict__ y) {
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
                const float *src = x + ((b * H + Y) * W + X) * 3;
#pragma unroll
                for (int ci = 0; ci < 3; ++ci) xin[ci * 9 + ky * 3 + kx] = in ? src[ci] : 0.f;
            }
    } else {
#pragma unroll
        for (int k = 0; k < KT; ++k) xin[k] = 0.f;
    }
    float *row = s + threadIdx.x * F_PITCH;
#pragma unroll
    for (int c4 = 0; c4 < CO / 4; ++c4) {
        float a[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float *wc = w + (4 * c4 + j) * KT;  // uniform over the block: scalar loads
            float v = 0.f;
#pragma unroll
            for (int k = 0; k < KT; ++k) v = fmaf(wc[k], xin[k], v);
            a[j] = bias ? v + bias[4 * c4 + j] : v;
        }
        *reinterpret_cast<float4 *>(row + 4 * c4) = make_float4(a[0], a[1], a[2], a[3]);
    }
    __syncthreads();
    // store: 256 pixels × 16 float4, consecutive threads -> consecutive float4 of the contiguous [pixel][64] output
#pragma unroll 4
    for (int k = 0; k < CO / 4; ++k) {
        const int idx = threadIdx.x + F_BLK * k, px = idx >> 4, c = 4 * (idx & 15);
        const long long q = p0 + px;
        if (q >= P) continue;
        float4 v = *reinterpret_cast<const float4 *>(s + px * F_PITCH + c);
        float *dst = y + q * CO + c;
        if (flags & ESR_DFIRST_ACC) {
            const float4 o = *reinterpret_cast<const float4 *>(dst);
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        if (flags & ESR_DFIRST_LRELU) {
            v.x = v.x > 0.f ? v.x : v.x * slope; v.y = v.y > 0.f ? v.y : v.y * slope;
            v.z = v.z > 0.f ? v.z : v.z * slope; v.w = v.w > 0.f ? v.w : v.w * slope;
        }
        if (flags & ESR_DFIRST_MASK) {
            const float4 mm = *reinterpret_cast<const float4 *>(m + q * CO + c);
            v.x *= lrelu_mask(mm.x, slope); v.y *= lrelu_mask(mm.y, slope);
            v.z *= lrelu_mask(mm.z, slope); v.w *= lrelu_mask(mm.w, slope);
        }
        *reinterpret_cast<float4 *>(dst) = v;
    }
}

// ---- backward --------------------------------------------------------------------------------------------------
// Block = 256 threads over 8 × 32-pixel output tiles (tile t = blockIdx.x + k·gridDim.x).  Per tile: the input on the
// tile + halo (10 × 34 pixels × 3) and, per 16-channel chunk, g' = gy · lrelu'(m) on the tile + halo in LDS.
//   input gradient (thread = tile pixel): gx[r][ci] = Σ_{ky,kx,co} w[co][ci][ky][kx] · g'[r − (ky − 1, kx − 1)][co]
//   weight / bias gradient (thread = (pixel group of 16, 4 channels of the chunk, 7 of the 27 (ci, tap) entries)):
//     dw[co][k] += Σ_p x[p + tap(k) − 1][ci(k)] · g'[p][co], db[co] += Σ_p g'[p][co] over its 16 pixels; the 16
//     pixel groups are added in group order at the end and the block writes its NW partial sums.
constexpr int B_TY = 8, B_TX = 32, B_HY = B_TY + 2, B_HX = B_TX + 2, B_HP = B_HY * B_HX;  // 340 halo pixels
constexpr int B_CC = 16, B_GP = B_CC + 4;                      // g' chunk channels, LDS pitch (floats)
constexpr int B_KB = 7;                                        // (ci, tap) entries per thread (4 groups: 7 7 7 6)
constexpr int B_RED = 16 * (B_CC * KT + B_CC);                 // one chunk's 16 pixel-group partials (floats)
constexpr int B_SG = B_HP * B_GP > B_RED ? B_HP * B_GP : B_RED;

__global__ __launch_bounds__(256) void dfirst_bwd_kernel(const float *__restrict__ x, const float *__restrict__ gy,
                                                         const float *__restrict__ m, float slope, int B, int H, int W,
                                                         const float *__restrict__ w, float *__restrict__ gx,
                                                         float *__restrict__ partial) {
    __shared__ __attribute__((aligned(16))) float sg[B_SG];
    __shared__ float sx[B_HP * 3];
    const int t = threadIdx.x;
    const int tiles_x = (W + B_TX - 1) / B_TX, tiles_y = (H + B_TY - 1) / B_TY;
    const long long ntiles = (long long)B * tiles_y * tiles_x;
    // weight-gradient role
    const int pg = t >> 4, cb = t & 3, kb = (t >> 2) & 3;
    float aw[4][4][B_KB], ab[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ab[c][j] = 0.f;
#pragma unroll
            for (int k = 0; k < B_KB; ++k) aw[c][j][k] = 0.f;
        }
    int xoff[B_KB];  // LDS offset (within sx, from a pixel's halo origin) of each of this thread's (ci, tap) entries
#pragma unroll
    for (int kk = 0; kk < B_KB; ++kk) {
        const int k = min(kb * B_KB + kk, KT - 1), ci = k / 9, tap = k - 9 * ci, ky = tap / 3, kx = tap - 3 * ky;
        xoff[kk] = (ky * B_HX + kx) * 3 + ci;
    }
    const int nk = min(B_KB, KT - kb * B_KB);  // entries of this thread (7, or 6 for the last group)
    const int ty = t >> 5, tx = t & 31;  // input-gradient role: this tile pixel
    for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int txi = (int)(tile % tiles_x);
        const long long r = tile / tiles_x;
        const int tyi = (int)(r % tiles_y);
        const long long b = r / tiles_y;
        const int y0 = tyi * B_TY, x0 = txi * B_TX;
        __syncthreads();  // the previous tile's LDS reads are done
        for (int i = t; partial && i < B_HP * 3; i += 256) {  // (x is read by the weight gradient only; may be NULL)
            const int hp = i / 3, ci = i - 3 * hp, hy = hp / B_HX, hx = hp - hy * B_HX;
            const int Y = y0 + hy - 1, X = x0 + hx - 1;
            sx[i] = (Y >= 0 && Y < H && X >= 0 && X < W) ? x[((b * H + Y) * W + X) * 3 + ci] : 0.f;
        }
        float ga[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (c) __syncthreads();  // the previous chunk's reads are done
            for (int i = t; i < B_HP * 4; i += 256) {
                const int hp = i >> 2, q = i & 3, hy = hp / B_HX, hx = hp - hy * B_HX;
                const int Y = y0 + hy - 1, X = x0 + hx - 1;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (Y >= 0 && Y < H && X >= 0 && X < W) {
                    const long long o = ((b * H + Y) * W + X) * CO + B_CC * c + 4 * q;
                    v = *reinterpret_cast<const float4 *>(gy + o);
                    if (m) {
                        const float4 mm = *reinterpret_cast<const float4 *>(m + o);
                        v.x *= lrelu_mask(mm.x, slope); v.y *= lrelu_mask(mm.y, slope);
                        v.z *= lrelu_mask(mm.z, slope); v.w *= lrelu_mask(mm.w, slope);
                    }
                }
                *reinterpret_cast<float4 *>(sg + hp * B_GP + 4 * q) = v;
            }
            __syncthreads();
            if (gx) {
#pragma unroll
                for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) {
                        const float *g = sg + ((ty + 2 - ky) * B_HX + tx + 2 - kx) * B_GP;
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const float4 g4 = *reinterpret_cast<const float4 *>(g + 4 * q);
                            const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const float *wc = w + (B_CC * c + 4 * q + j) * KT + ky * 3 + kx;  // uniform
#pragma unroll
                                for (int ci = 0; ci < 3; ++ci) ga[ci] = fmaf(wc[ci * 9], gv[j], ga[ci]);
                            }
                        }
                    }
            }
            if (partial) {
#pragma unroll 2
                for (int pl = 0; pl < 16; ++pl) {
                    const int pp = pg * 16 + pl, py = pp >> 5, px = pp & 31;
                    const float4 g4 = *reinterpret_cast<const float4 *>(sg + ((py + 1) * B_HX + px + 1) * B_GP + 4 * cb);
                    const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
                    const float *xs = sx + (py * B_HX + px) * 3;
#pragma unroll
                    for (int kk = 0; kk < B_KB; ++kk) {
                        const float xv = kk < nk ? xs[xoff[kk]] : 0.f;  // (the 27th slot of group 3: adds 0)
#pragma unroll
                        for (int j = 0; j < 4; ++j) aw[c][j][kk] = fmaf(xv, gv[j], aw[c][j][kk]);
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) ab[c][j] += gv[j];
                }
            }
        }
        if (gx) {
            const int Y = y0 + ty, X = x0 + tx;
            if (Y < H && X < W) {
                float *d = gx + ((b * H + Y) * W + X) * 3;
                d[0] = ga[0];
                d[1] = ga[1];
                d[2] = ga[2];
            }
        }
    }
    if (!partial) return;
    // the 16 pixel groups' sums, added in group order, one chunk at a time through LDS
    float *out = partial + (long long)blockIdx.x * NW;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        __syncthreads();
        float *red = sg + pg * (B_CC * KT + B_CC);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 4 * cb + j;  // channel within the chunk
#pragma unroll
            for (int kk = 0; kk < B_KB; ++kk) {
                const int k = kb * B_KB + kk;
                if (k < KT) red[co * KT + k] = aw[c][j][kk];
            }
            if (kb == 0) red[B_CC * KT + co] = ab[c][j];
        }
        __syncthreads();
        for (int e = t; e < B_CC * KT + B_CC; e += 256) {
            float v = sg[e];
            for (int g = 1; g < 16; ++g) v += sg[g * (B_CC * KT + B_CC) + e];
            if (e < B_CC * KT) {
                const int co = e / KT, k = e - KT * co;
                out[(B_CC * c + co) * KT + k] = v;
            } else {
                out[CO * KT + B_CC * c + (e - B_CC * KT)] = v;
            }
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
                       (hipStream_t)stream, x, P, H, W, w, bias, slope, flags, mask, y);
    return launched();
}

extern "C" int esr_dfirst_bwd_blocks(int32_t B, int32_t H, int32_t W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    const long long ntiles = (long long)B * ((H + B_TY - 1) / B_TY) * ((W + B_TX - 1) / B_TX);
    return (int)(ntiles < 512 ? ntiles : 512);
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
