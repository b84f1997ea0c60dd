// esr_train.hip — backward-pass kernels of the RRDB generator + CEM for gfx950 (training step, Z optimisation).
//
// The data gradient of a 3×3 conv is itself a 3×3 conv (rot180, in/out channels swapped) and runs on
// esr_conv3x3_fwd with repacked weights.  This file adds what has no forward counterpart:
//   esr_conv3x3_wgrad  weight (+bias) gradient: dW[tap][ci][co] = Σ_pixels in[p + tap][ci] · dout[p][co], a GEMM with
//                      K = pixels, on v_mfma_f32_32x32x2_f32 (exact fp32); split-K over pixel tiles into
//                      deterministic per-split partials, then esr_wgrad_reduce (fixed summation order, no atomics).
//   esr_lrelu_bwd      d *= (y > 0 ? 1 : 0.2) from the saved LeakyReLU output (block.py:10-23)
//   esr_axpby          y = a·x1 + b·x2 on channel slices of padded NHWC buffers (residual fan-in, block.py:96,235,270)
//   esr_sum2x2         adjoint of nearest ×2 upsampling (block.py:298)
//   esr_nchw_to_padded layout adapter between NCHW images and padded NHWC feature maps
//   esr_cem_adjoint    exact adjoint of the CEM stencils with replicate padding (CEMnet.py:149-162):
//                      for F(x)[o] = Σ_u w[u] x[clamp(s·o + c + u - p)] it gathers
//                      F^T(g)[k] = Σ_{(o,u): clamp(s·o + c + u - p) = k} w[u] g[o]   (2-D, separable clamp)
#include <hip/hip_runtime.h>
#include "esr_amd.h"
#include "esr_knobs.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

constexpr int NT = 256;
inline unsigned nblocks(long long n) { return (unsigned)((n + NT - 1) / NT); }

// value of channel c of a pixel record in the split-f16 layout (include/esr_amd.h: groups of 8 channels, 32 B =
// 8 × f16 hi then 8 × f16 lo); `rec` points at the pixel's first byte
__device__ __forceinline__ float split_at(const unsigned char *rec, int c) {
    const _Float16 *g = reinterpret_cast<const _Float16 *>(rec + (c >> 3) * 32);
    return (float)g[c & 7] + (float)g[8 + (c & 7)];
}
inline int launched() { return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH; }

// ---------------------------------------------------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------------------------------------------------
constexpr int WT_TH = 8, WT_TW = 32, WT_HY = WT_TH + 2, WT_HX = WT_TW + 2;
constexpr int WT_IP = 36;  // LDS pitch of a staged input pixel (32 channels)
constexpr int WT_DP = 68;  // LDS pitch of a staged output-gradient pixel (64 channels)
constexpr int WT_MAXP = 5; // (tap, co-tile) pairs per wave: 9 taps × 2 co-tiles over 4 waves

struct WgradParams {
    const float *in;
    int in_cp, cin, up2;
    const float *dout;
    int dout_cp, dout_coff, cout, cout_pad;
    int B, H, W, tiles_x, tiles_y, splits, cin_pad;
    float *partial;  // [splits][9*cin_pad*cout_pad + cout_pad]
    int dsplit;      // output gradient in the split-f16 layout (x3 kernel only)
    int dbg;         // wgrad3d diagnostic time split (ablation library only: g_wgrad3d_dbg)
};

__global__ __launch_bounds__(256, 1) void wgrad_kernel(WgradParams p) {
    __shared__ __attribute__((aligned(16))) float s_in[WT_HY * WT_HX * WT_IP];
    __shared__ __attribute__((aligned(16))) float s_d[WT_TH * WT_TW * WT_DP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ml = lane & 31;
    const int chunk = blockIdx.x % (p.cin_pad / 32);
    const int split = blockIdx.x / (p.cin_pad / 32);
    const int ntiles = p.B * p.tiles_y * p.tiles_x;
    const int t_begin = (int)((long long)ntiles * split / p.splits);
    const int t_end = (int)((long long)ntiles * (split + 1) / p.splits);
    const int nct = p.cout_pad / 32;
    const int npairs = 9 * nct;
    const int c0 = chunk * 32;
    const int kc = min(32, p.cin - c0);

    f32x16 acc[WT_MAXP];
#pragma unroll
    for (int i = 0; i < WT_MAXP; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    float bsum = 0.f;  // bias partial: thread (co = tid & 63) over pixels tid>>6 (+4)

    const int Hi = p.up2 ? p.H / 2 : p.H, Wi = p.up2 ? p.W / 2 : p.W;  // input grid
    for (int t = t_begin; t < t_end; ++t) {
        const int tx = t % p.tiles_x, ty = (t / p.tiles_x) % p.tiles_y, b = t / (p.tiles_x * p.tiles_y);
        const int y0 = ty * WT_TH, x0 = tx * WT_TW;
        __syncthreads();
        // input halo tile (output-grid coordinates, zero outside)
        for (int idx = tid; idx < WT_HY * WT_HX * 8; idx += 256) {
            const int px = idx >> 3, c4 = idx & 7;
            const int hy = px / WT_HX, hx = px - hy * WT_HX;
            const int Y = y0 + hy - 1, X = x0 + hx - 1;  // output-grid coords of this halo pixel
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (Y >= 0 && Y < p.H && X >= 0 && X < p.W && c4 * 4 < kc) {
                const int sy = p.up2 ? Y / 2 : Y, sx = p.up2 ? X / 2 : X;
                const float *src = p.in + (((long long)b * (Hi + 2) + sy + 1) * (Wi + 2) + sx + 1) * p.in_cp + c0 + c4 * 4;
                v = *reinterpret_cast<const f32x4 *>(src);
            }
            *reinterpret_cast<f32x4 *>(s_in + px * WT_IP + c4 * 4) = v;
        }
        // output-gradient tile
        for (int idx = tid; idx < WT_TH * WT_TW * 16; idx += 256) {
            const int px = idx >> 4, c4 = idx & 15;
            const int y = y0 + px / WT_TW, x = x0 + px % WT_TW;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (y < p.H && x < p.W && c4 * 4 < p.cout) {
                const float *src = p.dout + (((long long)b * (p.H + 2) + y + 1) * (p.W + 2) + x + 1) * p.dout_cp +
                                   p.dout_coff + c4 * 4;
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = (c4 * 4 + k < p.cout) ? src[k] : 0.f;
            }
            *reinterpret_cast<f32x4 *>(s_d + px * WT_DP + c4 * 4) = v;
        }
        __syncthreads();
        if (chunk == 0 && tid < 64 * 4)
            for (int px = tid >> 6; px < WT_TH * WT_TW; px += 4) bsum += s_d[px * WT_DP + (tid & 63)];
        // K loop: pixel pairs; lane half h takes pixel 2s+h
        for (int s = 0; s < WT_TH * WT_TW / 2; ++s) {
            const int px = 2 * s + hl;
            const int py = px / WT_TW, pxx = px % WT_TW;
#pragma unroll
            for (int i = 0; i < WT_MAXP; ++i) {
                const int pr = wave + 4 * i;
                if (pr >= npairs) break;
                const int tap = pr / nct, ct = pr - (pr / nct) * nct;
                const int hp = (py + tap / 3) * WT_HX + pxx + tap % 3;
                const float a = s_in[hp * WT_IP + ml];
                const float bb = s_d[px * WT_DP + ct * 32 + ml];
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc[i], 0, 0, 0);
            }
        }
    }
    // D layout: lane column j = co (ml), rows i = ci = (r&3) + 8*(r>>2) + 4*hl
    float *part = p.partial + (long long)split * (9LL * p.cin_pad * p.cout_pad + p.cout_pad);
#pragma unroll
    for (int i = 0; i < WT_MAXP; ++i) {
        const int pr = wave + 4 * i;
        if (pr >= npairs) break;
        const int tap = pr / nct, ct = pr - (pr / nct) * nct;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ci = c0 + (r & 3) + 8 * (r >> 2) + 4 * hl;
            part[((long long)tap * p.cin_pad + ci) * p.cout_pad + ct * 32 + ml] = acc[i][r];
        }
    }
    // bias partial (chunk-0 workgroups): reduce the 4 pixel-phase partials through LDS
    if (chunk == 0) {
        __syncthreads();
        s_d[tid] = bsum;
        __syncthreads();
        if (tid < p.cout_pad) {
            float v = 0.f;
            if (tid < 64) v = s_d[tid] + s_d[64 + tid] + s_d[128 + tid] + s_d[192 + tid];
            part[9LL * p.cin_pad * p.cout_pad + tid] = v;
        }
    }
}

// wgrad2: the same GEMM with 12 waves (3 per SIMD) instead of 4, so LDS and MFMA latencies of one wave hide behind
// the others.  Wave w owns the three taps of tap column tg = w % 3 (dy = 0..2, dx = tg) for one output-channel tile ct
// and one pixel class q (N = 32: 4 classes; N = 64: 2 channel tiles x 2 classes), i.e. 3 accumulators; per pixel pair
// it reads one output-gradient fragment (reused by its 3 taps) and one input fragment per tap.  LDS rows are unpadded
// (128 B per 32 channels: conflict-free for these lane patterns).  (Measured: 6-wave workgroups for N = 32, two per CU,
// were 10-15 % slower — the SIMDs hold 2 + 2 + 1 + 1 waves of one workgroup.)  The next pixel tile's global loads are
// issued into registers before the current tile is consumed.  The pixel classes are summed through LDS at the end
// (fixed order).  blockIdx is remapped so that the chunks of one split run on the same XCD and share its L2 for the
// output gradient.
constexpr int W2_IP = 32;  // LDS pitch of a staged input pixel (32 channels, no padding)

template <int NCT>
struct W2 {
    static constexpr int NWV = 12, NT = 64 * NWV, NQ = 4 / NCT;
    static constexpr int DP = 32 * NCT;  // LDS pitch of a staged output-gradient pixel
    static constexpr int IN_F = WT_HY * WT_HX * W2_IP, D_F = WT_TH * WT_TW * DP;
    static constexpr int IN_V4 = WT_HY * WT_HX * 8, D_V4 = WT_TH * WT_TW * 8 * NCT;
    static constexpr int IN_PT = 2 * ((IN_V4 / 2 + NT - 1) / NT), D_PT = (D_V4 + NT - 1) / NT;
};

template <int NCT, bool SPLIT>
__global__ __launch_bounds__(W2<NCT>::NT, 1) void wgrad2_kernel(WgradParams p) {
    using C = W2<NCT>;
    constexpr int NT_ = C::NT, NQ = C::NQ, DP = C::DP;
    static_assert(C::IN_V4 <= C::IN_PT * NT_, "input staging");
    __shared__ __attribute__((aligned(16))) float smem[C::IN_F + C::D_F];
    float *s_in = smem, *s_d = smem + C::IN_F;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ml = lane & 31;
    const int tg = wave % 3, r4 = wave / 3;
    const int ct = NCT == 2 ? (r4 & 1) : 0, q = NCT == 2 ? (r4 >> 1) : r4;
    const int nchunks = p.cin_pad / 32;
    const int total = nchunks * p.splits;
    // XCD-aware logical id: the hardware dispatches blockIdx round-robin over the 8 XCDs
    const int per_xcd = (total + 7) / 8;
    const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (L >= total) return;
    const int chunk = L % nchunks, split = L / nchunks;
    const int ntiles = p.B * p.tiles_y * p.tiles_x;
    const int t_begin = (int)((long long)ntiles * split / p.splits);
    const int t_end = (int)((long long)ntiles * (split + 1) / p.splits);
    const int c0 = chunk * 32;
    const int kc = min(32, p.cin - c0);
    const int Hi = p.up2 ? p.H / 2 : p.H, Wi = p.up2 ? p.W / 2 : p.W;
    const bool vec_d = ((p.dout_cp | p.dout_coff) & 3) == 0;  // 16-B aligned output-gradient pixels

    f32x16 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    float bsum = 0.f;

    f32x4 rin[C::IN_PT], rd[C::D_PT];
    auto load_tile = [&](int t) {
        const int tx = t % p.tiles_x, ty = (t / p.tiles_x) % p.tiles_y, b = t / (p.tiles_x * p.tiles_y);
        const int y0 = ty * WT_TH, x0 = tx * WT_TW;
        if (SPLIT) {
            // one 8-channel group (32 B: hi[8], lo[8]) per item, 4 groups per pixel, two register quads per item
#pragma unroll
            for (int k = 0; k < C::IN_PT / 2; ++k) {
                const int idx = tid + k * NT_;
                const int px = idx >> 2, g = idx & 3;
                const int hy = px / WT_HX, hx = px - hy * WT_HX;
                const int Y = y0 + hy - 1, X = x0 + hx - 1;
                f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
                if (idx < C::IN_V4 / 2 && Y >= 0 && Y < p.H && X >= 0 && X < p.W && g * 8 < kc) {
                    const int sy = p.up2 ? Y / 2 : Y, sx = p.up2 ? X / 2 : X;
                    const f16x8 *src = reinterpret_cast<const f16x8 *>(
                        reinterpret_cast<const unsigned char *>(p.in) +
                        ((((long long)b * (Hi + 2) + sy + 1) * (Wi + 2) + sx + 1) * p.in_cp + c0 + g * 8) * 4);
                    const f16x8 hi = src[0], lo = src[1];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v0[e] = (float)hi[e] + (float)lo[e];
                        v1[e] = (float)hi[4 + e] + (float)lo[4 + e];
                    }
                }
                rin[2 * k] = v0;
                rin[2 * k + 1] = v1;
            }
        } else {
#pragma unroll
            for (int k = 0; k < C::IN_PT; ++k) {
                const int idx = tid + k * NT_;
                const int px = idx >> 3, c4 = idx & 7;
                const int hy = px / WT_HX, hx = px - hy * WT_HX;
                const int Y = y0 + hy - 1, X = x0 + hx - 1;
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
                if (idx < C::IN_V4 && Y >= 0 && Y < p.H && X >= 0 && X < p.W && c4 * 4 < kc) {
                    const int sy = p.up2 ? Y / 2 : Y, sx = p.up2 ? X / 2 : X;
                    v = *reinterpret_cast<const f32x4 *>(
                        p.in + (((long long)b * (Hi + 2) + sy + 1) * (Wi + 2) + sx + 1) * p.in_cp + c0 + c4 * 4);
                }
                rin[k] = v;
            }
        }
#pragma unroll
        for (int k = 0; k < C::D_PT; ++k) {
            const int idx = tid + k * NT_;
            const int px = idx / (8 * NCT), c4 = idx % (8 * NCT);
            const int y = y0 + (px >> 5), x = x0 + (px & 31);
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (idx < C::D_V4 && y < p.H && x < p.W && c4 * 4 < p.cout) {
                const float *src = p.dout + (((long long)b * (p.H + 2) + y + 1) * (p.W + 2) + x + 1) * p.dout_cp +
                                   p.dout_coff + c4 * 4;
                if (vec_d && c4 * 4 + 4 <= p.cout) {
                    v = *reinterpret_cast<const f32x4 *>(src);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = (c4 * 4 + e < p.cout) ? src[e] : 0.f;
                }
            }
            rd[k] = v;
        }
    };
    auto store_tile = [&]() {
        if (SPLIT) {
#pragma unroll
            for (int k = 0; k < C::IN_PT / 2; ++k) {
                const int idx = tid + k * NT_;
                if (idx < C::IN_V4 / 2) {
                    float *dst = s_in + (idx >> 2) * W2_IP + (idx & 3) * 8;
                    *reinterpret_cast<f32x4 *>(dst) = rin[2 * k];
                    *reinterpret_cast<f32x4 *>(dst + 4) = rin[2 * k + 1];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < C::IN_PT; ++k) {
                const int idx = tid + k * NT_;
                if (idx < C::IN_V4) *reinterpret_cast<f32x4 *>(s_in + (idx >> 3) * W2_IP + (idx & 7) * 4) = rin[k];
            }
        }
#pragma unroll
        for (int k = 0; k < C::D_PT; ++k) {
            const int idx = tid + k * NT_;
            if (idx < C::D_V4) *reinterpret_cast<f32x4 *>(s_d + idx * 4) = rd[k];  // [pixel][DP] is dense
        }
    };

    // bias partial (chunk-0 workgroups): thread (channel tid % DP, pixel phase tid / DP) for tid < 256
    constexpr int BPH = 256 / DP;
    if (t_begin < t_end) load_tile(t_begin);
    for (int t = t_begin; t < t_end; ++t) {
        __syncthreads();
        store_tile();
        __syncthreads();
        if (t + 1 < t_end) load_tile(t + 1);
        if (chunk == 0 && tid < 256)
            for (int px = tid / DP; px < WT_TH * WT_TW; px += BPH) bsum += s_d[px * DP + tid % DP];
        // pixel pairs s = NQ*k + q; lane half hl takes pixel 2s + hl
#pragma unroll 4
        for (int k = 0; k < WT_TH * WT_TW / (2 * NQ); ++k) {
            const int px = 2 * (NQ * k + q) + hl;
            const int py = px >> 5, pxx = px & 31;
            const float bb = s_d[px * DP + ct * 32 + ml];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const float a = s_in[((py + j) * WT_HX + pxx + tg) * W2_IP + ml];
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc[j], 0, 0, 0);
            }
        }
    }
    // sum the pixel classes into class 0 (fixed order 1, 2, ...), through LDS
    constexpr int PER_WAVE = 3 * 16 * 64;
    static_assert(3 * NCT * PER_WAVE <= C::IN_F + C::D_F, "class reduction does not fit in LDS");
    const int slot = tg * NCT + ct;
    for (int r = 1; r < NQ; ++r) {
        __syncthreads();
        if (q == r) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) smem[slot * PER_WAVE + (j * 16 + e) * 64 + lane] = acc[j][e];
        }
        __syncthreads();
        if (q == 0) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[j][e] += smem[slot * PER_WAVE + (j * 16 + e) * 64 + lane];
        }
    }
    float *part = p.partial + (long long)split * (9LL * p.cin_pad * p.cout_pad + p.cout_pad);
    if (q == 0) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int tap = 3 * j + tg;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int ci = c0 + (e & 3) + 8 * (e >> 2) + 4 * hl;
                part[((long long)tap * p.cin_pad + ci) * p.cout_pad + ct * 32 + ml] = acc[j][e];
            }
        }
    }
    if (chunk == 0) {
        __syncthreads();
        if (tid < 256) smem[tid] = bsum;
        __syncthreads();
        if (tid < p.cout_pad) {
            float v = 0.f;
            for (int ph = 0; ph < BPH; ++ph) v += smem[ph * DP + tid];
            part[9LL * p.cin_pad * p.cout_pad + tid] = v;
        }
    }
}

// wgrad3 (x3): the same GEMM on v_mfma_f32_32x32x16_f16 in the split-f16 scheme of the forward — products
// a_hi·b_hi + a_hi·b_lo + a_lo·b_hi, fp32 accumulation.  A = the input activations, already split by the x3 forward
// (f16 hi/lo groups of 8 channels); B = the output gradient, fp32 in memory, split here per pixel tile after scaling
// by 2^e (e from the tile's max |dout|, so that its largest element lands in [2^13, 2^14) and the lo parts stay far
// above f16's subnormal range).  The accumulators live in the scale of the current tile: on a scale change they are
// multiplied by 2^(e_new - e_old) (v_ldexp: exact), and by 2^-e at the end — so the result equals the unscaled sum
// up to the products' rounding.  The bias gradient is summed from the fp32 values (exact fp32).
// K = pixels: both operands are read with ds_read_b64_tr_b16 from pixel-major LDS images (128 B per pixel and 32
// channels: the global split record as it stands), 4 consecutive pixels × 16 channels per 16-lane group, so a tap's
// pixel shift is only a different row address.  Bank conflicts: pixels p and p+2 share their bank set (128-B rows),
// so pixel p stores its hi and lo halves swapped when (p >> 1) & 1 — the 4 pixels × 32 channels of one read then
// cover the 64 banks exactly.  Waves as in wgrad2 (tap column tg, output-channel tile ct, pixel class q; 3 taps per
// wave), 12 waves, next tile's global loads in registers while the current one is consumed.
template <int NCT>
struct W3 {
    static constexpr int NWV = 12, NT = 64 * NWV, NQ = 4 / NCT;
    static constexpr int IN_PX = WT_HY * WT_HX;                 // halo pixels
    static constexpr int IN_B = IN_PX * 128;                    // input image bytes
    static constexpr int D_B = WT_TH * WT_TW * 128;             // one output-channel tile's image bytes
    static constexpr int IN_IT = IN_PX * 8;                     // 16-B items of the input tile
    static constexpr int IN_PT = (IN_IT + NT - 1) / NT;
    static constexpr int D_V4 = WT_TH * WT_TW * 8 * NCT;        // fp32 quads of the output-gradient tile
    static constexpr int D_PT = (D_V4 + NT - 1) / NT;
    static constexpr int RED_B = 2 * NWV * 4;                   // per-wave max |dout|, double-buffered
    static constexpr int LDS_B = IN_B + NCT * D_B + RED_B;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 tr_read(const unsigned char *lds, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(lds + byte_off));
}
__device__ __forceinline__ f16x8 cat8(s16x4 a, s16x4 b) {
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NCT>
__global__ __launch_bounds__(W3<NCT>::NT, 1) void wgrad3_kernel(WgradParams p) {
    using C = W3<NCT>;
    constexpr int NT_ = C::NT, NQ = C::NQ;
    static_assert(NT_ % (8 * NCT) == 0, "a thread's output-gradient channel quad must not change across items");
    __shared__ __attribute__((aligned(16))) unsigned char smem[C::LDS_B];
    unsigned char *s_in = smem, *s_d = smem + C::IN_B;
    float *s_red = reinterpret_cast<float *>(smem + C::IN_B + NCT * C::D_B);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5;
    const int tg = wave % 3, r4 = wave / 3;
    const int ct = NCT == 2 ? (r4 & 1) : 0, q = NCT == 2 ? (r4 >> 1) : r4;
    const int nchunks = p.cin_pad / 32;
    const int total = nchunks * p.splits;
    const int per_xcd = (total + 7) / 8;
    const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (L >= total) return;
    const int chunk = L % nchunks, split = L / nchunks;
    const int ntiles = p.B * p.tiles_y * p.tiles_x;
    const int t_begin = (int)((long long)ntiles * split / p.splits);
    const int t_end = (int)((long long)ntiles * (split + 1) / p.splits);
    const int c0 = chunk * 32;
    const int kc = min(32, p.cin - c0);
    const int Hi = p.up2 ? p.H / 2 : p.H, Wi = p.up2 ? p.W / 2 : p.W;
    const bool vec_d = ((p.dout_cp | p.dout_coff) & 3) == 0;
    const int my_c4 = tid % (8 * NCT);  // this thread's output-gradient channel quad (fixed, see static_assert)

    // transposed-read lane roles: group i16 = lane & 15 supplies row (pixel) rq = i16 >> 2, channel block 4·(i16 & 3)
    // of the 16 channels 16·((lane >> 4) & 1) ...; the half hl takes K rows 8·hl ...
    const int i16 = lane & 15, rq = i16 >> 2;
    const int chb = 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);      // first channel of the lane's 4-channel block
    const int ch_off = (chb >> 3) * 32 + (chb & 4) * 2;           // its byte offset in a 128-B pixel record (hi)

    f32x16 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    f32x4 bacc = {0.f, 0.f, 0.f, 0.f};
    int e_cur = 0;

    f32x4 rin[C::IN_PT], rd[C::D_PT];
    auto load_tile = [&](int t) {
        const int tx = t % p.tiles_x, ty = (t / p.tiles_x) % p.tiles_y, b = t / (p.tiles_x * p.tiles_y);
        const int y0 = ty * WT_TH, x0 = tx * WT_TW;
#pragma unroll
        for (int k = 0; k < C::IN_PT; ++k) {
            const int idx = tid + k * NT_;
            const int px = idx >> 3, part = idx & 7;  // part = 2·group + (0 hi | 1 lo)
            const int hy = px / WT_HX, hx = px - hy * WT_HX;
            const int Y = y0 + hy - 1, X = x0 + hx - 1;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (idx < C::IN_IT && Y >= 0 && Y < p.H && X >= 0 && X < p.W && (part >> 1) * 8 < kc) {
                const int sy = p.up2 ? Y / 2 : Y, sx = p.up2 ? X / 2 : X;
                v = *reinterpret_cast<const f32x4 *>(
                    reinterpret_cast<const unsigned char *>(p.in) +
                    ((((long long)b * (Hi + 2) + sy + 1) * (Wi + 2) + sx + 1) * p.in_cp + c0) * 4 + part * 16);
            }
            rin[k] = v;
        }
#pragma unroll
        for (int k = 0; k < C::D_PT; ++k) {
            const int idx = tid + k * NT_;
            const int px = idx / (8 * NCT), c4 = idx % (8 * NCT);
            const int y = y0 + (px >> 5), x = x0 + (px & 31);
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (idx < C::D_V4 && y < p.H && x < p.W && c4 * 4 < p.cout) {
                const long long pix = ((long long)b * (p.H + 2) + y + 1) * (p.W + 2) + x + 1;
                if (p.dsplit) {  // 4 channels = half an 8-channel group: f16 hi[4] at +0, lo[4] at +16
                    const unsigned char *g = reinterpret_cast<const unsigned char *>(p.dout) +
                                             (pix * p.dout_cp + p.dout_coff + (c4 >> 1) * 8) * 4 + (c4 & 1) * 8;
                    const f16x4 h = *reinterpret_cast<const f16x4 *>(g), l = *reinterpret_cast<const f16x4 *>(g + 16);
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = (float)h[e] + (float)l[e];
                } else {
                    const float *src = p.dout + pix * p.dout_cp + p.dout_coff + c4 * 4;
                    if (vec_d && c4 * 4 + 4 <= p.cout) {
                        v = *reinterpret_cast<const f32x4 *>(src);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = (c4 * 4 + e < p.cout) ? src[e] : 0.f;
                    }
                }
            }
            rd[k] = v;
        }
    };
    // max |dout| of the tile in registers: per wave (lane shuffles), then per workgroup through s_red[slot]
    auto publish_max = [&](int slot) {
        float m = 0.f;
#pragma unroll
        for (int k = 0; k < C::D_PT; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) m = fmaxf(m, fabsf(rd[k][e]));
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) m = fmaxf(m, __shfl_xor(m, s));
        if (lane == 0) s_red[slot * C::NWV + wave] = m;
    };
    auto store_tile = [&](float scale) {
#pragma unroll
        for (int k = 0; k < C::IN_PT; ++k) {
            const int idx = tid + k * NT_;
            if (idx < C::IN_IT) {
                const int px = idx >> 3, part = idx & 7;
                const int sw = ((px >> 1) & 1);  // hi/lo swap of pixel px
                *reinterpret_cast<f32x4 *>(s_in + px * 128 + (part >> 1) * 32 + ((part & 1) ^ sw) * 16) = rin[k];
            }
        }
#pragma unroll
        for (int k = 0; k < C::D_PT; ++k) {
            const int idx = tid + k * NT_;
            if (idx < C::D_V4) {
                const int px = idx / (8 * NCT), c4 = idx % (8 * NCT);
                const int cti = c4 >> 3, cq = c4 & 7;  // channel tile, quad within it
                f16x4 h, l;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = rd[k][e] * scale;
                    h[e] = (_Float16)x;
                    l[e] = (_Float16)(x - (float)h[e]);
                }
                const int sw = ((px >> 1) & 1);
                unsigned char *rec = s_d + cti * C::D_B + px * 128 + (cq >> 1) * 32 + (cq & 1) * 8;
                *reinterpret_cast<f16x4 *>(rec + sw * 16) = h;
                *reinterpret_cast<f16x4 *>(rec + (sw ^ 1) * 16) = l;
            }
        }
    };
    // byte offset of the lane's hi (lo = hi_or_lo 1) 4-channel block in pixel record px of an image
    auto rec_off = [&](int px, int lo) { return px * 128 + ch_off + ((lo ^ ((px >> 1) & 1)) << 4); };

    if (t_begin < t_end) {
        load_tile(t_begin);
        publish_max(0);
    }
    for (int t = t_begin; t < t_end; ++t) {
        __syncthreads();
        float m = 0.f;
#pragma unroll
        for (int w = 0; w < C::NWV; ++w) m = fmaxf(m, s_red[((t - t_begin) & 1) * C::NWV + w]);
        int e_new = e_cur;
        if (m > 0.f && m <= 3.4e38f) {  // a finite nonzero tile max; NaN / inf propagate unscaled
            int ex;
            frexpf(m, &ex);  // m < 2^ex
            e_new = 14 - ex;
        }
        if (e_new != e_cur) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[j][r] = ldexpf(acc[j][r], e_new - e_cur);
            e_cur = e_new;
        }
        if (chunk == 0) {
#pragma unroll
            for (int k = 0; k < C::D_PT; ++k)
                if (tid + k * NT_ < C::D_V4) bacc += rd[k];
        }
        store_tile(ldexpf(1.f, e_cur));
        __syncthreads();
        if (t + 1 < t_end) load_tile(t + 1);
        const unsigned char *img_d = s_d + ct * C::D_B;
#pragma unroll 2
        for (int kk = 0; kk < 16 / NQ; ++kk) {
            const int kb = NQ * kk + q;             // K block: 16 pixels of tile row kb >> 1
            const int py = kb >> 1, px0 = 16 * (kb & 1) + 8 * hl + rq;
            const int dp = py * WT_TW + px0;        // output-gradient pixel of K rows 8hl + rq (+4)
            const f16x8 bh = cat8(tr_read(img_d, rec_off(dp, 0)), tr_read(img_d, rec_off(dp + 4, 0)));
            const f16x8 bl = cat8(tr_read(img_d, rec_off(dp, 1)), tr_read(img_d, rec_off(dp + 4, 1)));
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int ip = (py + j) * WT_HX + px0 + tg;
                const f16x8 ah = cat8(tr_read(s_in, rec_off(ip, 0)), tr_read(s_in, rec_off(ip + 4, 0)));
                const f16x8 al = cat8(tr_read(s_in, rec_off(ip, 1)), tr_read(s_in, rec_off(ip + 4, 1)));
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[j], 0, 0, 0);
            }
        }
        if (t + 1 < t_end) publish_max((t + 1 - t_begin) & 1);
    }
    // back to the unscaled domain, then sum the pixel classes into class 0 (fixed order 1, 2, ...) through LDS
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = ldexpf(acc[j][r], -e_cur);
    constexpr int PER_WAVE = 3 * 16 * 64;
    static_assert(3 * NCT * PER_WAVE * 4 <= C::LDS_B, "class reduction does not fit in LDS");
    float *red = reinterpret_cast<float *>(smem);
    const int slot = tg * NCT + ct;
    for (int r = 1; r < NQ; ++r) {
        __syncthreads();
        if (q == r) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) red[slot * PER_WAVE + (j * 16 + e) * 64 + lane] = acc[j][e];
        }
        __syncthreads();
        if (q == 0) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[j][e] += red[slot * PER_WAVE + (j * 16 + e) * 64 + lane];
        }
    }
    float *part = p.partial + (long long)split * (9LL * p.cin_pad * p.cout_pad + p.cout_pad);
    if (q == 0) {
        const int ml = lane & 31;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int tap = 3 * j + tg;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int ci = c0 + (e & 3) + 8 * (e >> 2) + 4 * hl;
                part[((long long)tap * p.cin_pad + ci) * p.cout_pad + ct * 32 + ml] = acc[j][e];
            }
        }
    }
    if (chunk == 0) {  // bias: threads with the same channel quad, summed in thread order
        __syncthreads();
        reinterpret_cast<f32x4 *>(smem)[tid] = bacc;
        __syncthreads();
        if (tid < p.cout_pad) {
            const float *b4 = reinterpret_cast<const float *>(smem);
            float v = 0.f;
            for (int th = tid / 4; th < NT_; th += 8 * NCT) v += b4[th * 4 + (tid & 3)];
            part[9LL * p.cin_pad * p.cout_pad + tid] = v;
        }
    }
}

// wgrad3d: wgrad3 for an output gradient that is already split-f16 (dsplit: the x3 backward's residual-block
// gradients, values S·g at one scale S per pass, esr_grad_amax).  Both operands are then bit copies of global
// records, so both tiles go HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR staging, no per-tile max or
// rescale, no VALU split) into two LDS stages — tile t+1 is in flight while tile t is consumed, one barrier per tile.
// LDS images, swizzle (applied on the DMA source address: the destination of a DMA is lane-linear) and wave roles are
// wgrad3's, and so are the products (three f16 MFMAs per product on the stored f16 pieces; their scale is S, not a
// per-tile 2^e — both powers of two).  N = 64 (two channel tiles) takes 4-row pixel tiles so that two stages fit.
// The bias gradient is summed from the LDS image (hi + lo) by the chunk-0 workgroups.
template <int NCT, int TH>
struct W3D {
    static constexpr int NWV = 12, NT = 64 * NWV, NQ = 4 / NCT;
    static constexpr int HY = TH + 2, HX = WT_TW + 2, IN_PX = HY * HX, D_PX = TH * WT_TW;
    static constexpr int IN_PC = (IN_PX + 7) / 8, D_PC = D_PX / 8;  // 1-KB pieces (8 records of 128 B)
    static constexpr int IN_B = IN_PC * 1024, D_B = D_PC * 1024;
    static constexpr int STAGE = IN_B + NCT * D_B;
    static constexpr int PIECES = IN_PC + NCT * D_PC;
    static constexpr int KP = (PIECES + NWV - 1) / NWV;  // DMA wave-instructions per wave and tile
    static constexpr int LDS_B = 2 * STAGE;
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glob_void;
__device__ __attribute__((aligned(16))) unsigned char g_wzero[64];  // zero page: the DMA source of absent records

template <int NCT, int TH, int KU = 4>  // KU: unroll of the K-block loop (4 = full; A/B: esr_wgrad3d_set_unroll)
__global__ __launch_bounds__((W3D<NCT, TH>::NT), 1) void wgrad3d_kernel(WgradParams p) {
    using C = W3D<NCT, TH>;
    constexpr int NT_ = C::NT, NQ = C::NQ;
    static_assert(C::LDS_B <= 160 * 1024, "two stages per CU");
    static_assert(3 * NCT * 3 * 16 * 64 * 4 <= C::LDS_B && NT_ * 4 <= C::LDS_B, "reductions fit in LDS");
    __shared__ __attribute__((aligned(1024))) unsigned char smem[C::LDS_B];
    const int tid = threadIdx.x, lane = tid & 63, hl = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int tg = wave % 3, r4 = wave / 3;
    const int ct = NCT == 2 ? (r4 & 1) : 0, q = NCT == 2 ? (r4 >> 1) : r4;
    const int nchunks = p.cin_pad / 32;
    const int total = nchunks * p.splits;
    const int per_xcd = (total + 7) / 8;
    const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (L >= total) return;
    const int chunk = L % nchunks, split = L / nchunks;
    const int ntiles = p.B * p.tiles_y * p.tiles_x;
    const int t_begin = (int)((long long)ntiles * split / p.splits);
    const int t_end = (int)((long long)ntiles * (split + 1) / p.splits);
    const int c0 = chunk * 32;
    const int kg = (min(32, p.cin - c0) + 7) >> 3;  // 8-channel groups present in this chunk
    const int Hi = p.up2 ? p.H / 2 : p.H, Wi = p.up2 ? p.W / 2 : p.W;
    const unsigned char *gin = reinterpret_cast<const unsigned char *>(p.in);
    const unsigned char *gd = reinterpret_cast<const unsigned char *>(p.dout);
    const int drec = lane >> 3, slot = lane & 7, grp = slot >> 1;  // lane -> record of a piece, 16-B slot, group

    // DMA of tile t into stage stg: piece pc = wave + 12 i; LDS byte pc·1024 + 16·lane = record 8 pc + drec, slot;
    // the slot's logical half is (slot & 1) ^ swap(record), so the source half is chosen accordingly
    auto dma_tile = [&](int t, int stg) {
        const int tx = t % p.tiles_x, ty = (t / p.tiles_x) % p.tiles_y, b = t / (p.tiles_x * p.tiles_y);
        const int y0 = ty * TH, x0 = tx * WT_TW;
        unsigned char *base = smem + stg * C::STAGE;
#pragma unroll
        for (int i = 0; i < C::KP; ++i) {
            const int pc = wave + C::NWV * i;
            if (pc >= C::PIECES) break;
            const void *src = g_wzero;
            if (pc < C::IN_PC) {
                const int r = 8 * pc + drec;
                const int hy = r / C::HX, hx = r - hy * C::HX;
                const int Y = y0 + hy - 1, X = x0 + hx - 1;
                const int half = (slot & 1) ^ ((r >> 1) & 1);
                if (r < C::IN_PX && Y >= 0 && Y < p.H && X >= 0 && X < p.W && grp < kg) {
                    const int sy = p.up2 ? Y / 2 : Y, sx = p.up2 ? X / 2 : X;
                    src = gin + ((((long long)b * (Hi + 2) + sy + 1) * (Wi + 2) + sx + 1) * p.in_cp + c0) * 4 +
                          grp * 32 + half * 16;
                }
            } else {
                const int pd = pc - C::IN_PC, cti = pd / C::D_PC, r = 8 * (pd - cti * C::D_PC) + drec;
                const int y = y0 + (r >> 5), x = x0 + (r & 31);
                const int half = (slot & 1) ^ ((r >> 1) & 1);
                if (y < p.H && x < p.W && cti * 32 + grp * 8 < p.cout) {
                    const long long pix = ((long long)b * (p.H + 2) + y + 1) * (p.W + 2) + x + 1;
                    src = gd + (pix * p.dout_cp + p.dout_coff + cti * 32 + grp * 8) * 4 + half * 16;
                }
            }
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(base + pc * 1024), 16, 0, 0);
        }
    };

    // transposed-read lane roles as wgrad3
    const int i16 = lane & 15, rq = i16 >> 2;
    const int chb = 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
    const int ch_off = (chb >> 3) * 32 + (chb & 4) * 2;
    auto rec_off = [&](int px, int lo) { return px * 128 + ch_off + ((lo ^ ((px >> 1) & 1)) << 4); };
    // bias (chunk 0): thread -> channel bc of the 32·NCT, pixels bp0, bp0 + BST, ... of the tile
    constexpr int BST = NT_ / (32 * NCT);
    const int bc = tid % (32 * NCT), bp0 = tid / (32 * NCT);
    const int b_off = (bc >> 5) * C::D_B + ((bc & 31) >> 3) * 32 + (bc & 7) * 2;
    float bsum = 0.f;

    f32x16 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

#ifdef ESR_X3_EXPERIMENTS
    const int dbg = p.dbg;  // g_wgrad3d_dbg: 1 LDS-DMA of the first tile only, 2 no fragment reads / MFMAs
#else
    constexpr int dbg = 0;
#endif
    if (t_begin < t_end) dma_tile(t_begin, 0);
    for (int t = t_begin; t < t_end; ++t) {
        const int stg = (t - t_begin) & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile t are in LDS
        __syncthreads();  // ... every wave's; and every wave is done reading stage stg ^ 1 (tile t - 1)
        if (t + 1 < t_end && !(dbg & 1)) dma_tile(t + 1, stg ^ 1);
        const unsigned char *s_in = smem + stg * C::STAGE, *s_d = s_in + C::IN_B;
        if (chunk == 0) {
            for (int px = bp0; px < C::D_PX; px += BST) {
                const unsigned char *rc = s_d + b_off + px * 128;
                const int sw = (px >> 1) & 1;
                bsum += (float)*reinterpret_cast<const _Float16 *>(rc + (sw << 4)) +
                        (float)*reinterpret_cast<const _Float16 *>(rc + ((sw ^ 1) << 4));
            }
        }
        const unsigned char *img_d = s_d + ct * C::D_B;
        if (dbg & 2) continue;
#pragma unroll KU
        for (int kk = 0; kk < 2 * TH / NQ; ++kk) {
            const int kb = NQ * kk + q;             // K block: 16 pixels of tile row kb >> 1
            const int py = kb >> 1, px0 = 16 * (kb & 1) + 8 * hl + rq;
            const int dp = py * WT_TW + px0;
            const f16x8 bh = cat8(tr_read(img_d, rec_off(dp, 0)), tr_read(img_d, rec_off(dp + 4, 0)));
            const f16x8 bl = cat8(tr_read(img_d, rec_off(dp, 1)), tr_read(img_d, rec_off(dp + 4, 1)));
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int ip = (py + j) * C::HX + px0 + tg;
                const f16x8 ah = cat8(tr_read(s_in, rec_off(ip, 0)), tr_read(s_in, rec_off(ip + 4, 0)));
                const f16x8 al = cat8(tr_read(s_in, rec_off(ip, 1)), tr_read(s_in, rec_off(ip + 4, 1)));
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[j], 0, 0, 0);
            }
        }
    }
    // sum the pixel classes into class 0 (fixed order 1, 2, ...) through LDS, as wgrad3
    constexpr int PER_WAVE = 3 * 16 * 64;
    float *red = reinterpret_cast<float *>(smem);
    const int rslot = tg * NCT + ct;
    for (int r = 1; r < NQ; ++r) {
        __syncthreads();
        if (q == r) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) red[rslot * PER_WAVE + (j * 16 + e) * 64 + lane] = acc[j][e];
        }
        __syncthreads();
        if (q == 0) {
#pragma unroll
            for (int j = 0; j < 3; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[j][e] += red[rslot * PER_WAVE + (j * 16 + e) * 64 + lane];
        }
    }
    float *part = p.partial + (long long)split * (9LL * p.cin_pad * p.cout_pad + p.cout_pad);
    if (q == 0) {
        const int ml = lane & 31;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const int tap = 3 * j + tg;
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int ci = c0 + (e & 3) + 8 * (e >> 2) + 4 * hl;
                part[((long long)tap * p.cin_pad + ci) * p.cout_pad + ct * 32 + ml] = acc[j][e];
            }
        }
    }
    if (chunk == 0) {  // bias: the threads of one channel, summed in thread order
        __syncthreads();
        red[tid] = bsum;
        __syncthreads();
        if (tid < p.cout_pad) {
            float v = 0.f;
            for (int th = tid; th < NT_; th += 32 * NCT) v += red[th];
            part[9LL * p.cin_pad * p.cout_pad + tid] = v;
        }
    }
}



// Gradient scale of the x3 backward (esr_grad_amax): S = 2^(11 - ex) for max|g| < 2^ex, so the largest scaled
// element lies in [2^10, 2^11) (headroom 2^5 below the f16 range for growth through a residual block); 1 for an
// all-zero or non-finite max (a NaN / inf propagates unscaled).
__device__ __forceinline__ float gscale_of(const unsigned *amax) {
    if (!amax) return 1.f;
    const float m = __uint_as_float(*amax);
    if (!(m > 0.f) || !(m <= 3.4e38f)) return 1.f;
    int ex;
    frexpf(m, &ex);
    return ldexpf(1.f, 11 - ex);
}

// Each workgroup: 32 consecutive outputs × 8 slices of the splits; a slice is summed in split order, then the 8
// slice sums in slice order (fixed order: deterministic), so a reduction over ~100 splits runs with 8× the
// threads of a one-thread-per-output loop.
constexpr int RED_O = 32, RED_S = NT / RED_O;
__global__ void wgrad_reduce_kernel(const float *partial, int splits, long long n, float scale, float *out,
                                    const unsigned *amax, long long n_w = -1, float scale_b = 0.f) {
    __shared__ float sl[RED_S][RED_O];
    const int o = threadIdx.x % RED_O, q = threadIdx.x / RED_O;
    const long long i = (long long)blockIdx.x * RED_O + o;
    const int k0 = splits * q / RED_S, k1 = splits * (q + 1) / RED_S;
    float s = 0.f;
    if (i < n)
        for (int k = k0; k < k1; ++k) s += partial[(long long)k * n + i];
    sl[q][o] = s;
    __syncthreads();
    if (q == 0 && i < n) {
        float t = sl[0][o];
        for (int r = 1; r < RED_S; ++r) t += sl[r][o];
        const float sc = (n_w >= 0 && i >= n_w) ? scale_b : scale;  // entries past n_w: the bias gradients
        out[i] = amax ? (sc * t) / gscale_of(amax) : sc * t;
    }
}

// max |x| over a C-channel fp32 slice, OR-ed into *amax as float bits (non-negative floats order as unsigned ints)
// max |x| over a padded NHWC channel slice.  A block walks whole image rows (blockIdx.x + k·gridDim.x over the B·H
// rows), each row's W × C slice with 16-B loads where the slice is 4-aligned: the index math is per row, not per
// element (the per-element 64-bit divisions held it at ~0.5 TB/s, 120 µs per config-5 trunk gradient).
__global__ void grad_amax_kernel(const float *x, int cp, int coff, int C, int B, int H, int W, unsigned *amax) {
    __shared__ float red[NT / 64];
    float m = 0.f;
    const bool v4 = (C % 4 == 0) && (coff % 4 == 0) && (cp % 4 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15) == 0);
    const int C4 = C / 4;
    for (long long row = blockIdx.x; row < (long long)B * H; row += gridDim.x) {
        const long long b = row / H, y = row - b * H;
        const float *base = x + ((b * (H + 2) + y + 1) * (W + 2) + 1) * cp + coff;
        if (v4) {
            for (int k = threadIdx.x; k < W * C4; k += NT) {
                const int xx = k / C4, c4 = k - xx * C4;
                const f32x4 v = *reinterpret_cast<const f32x4 *>(base + (long long)xx * cp + 4 * c4);
                m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
            }
        } else {
            for (int k = threadIdx.x; k < W * C; k += NT) {
                const int xx = k / C, c = k - xx * C;
                m = fmaxf(m, fabsf(base[(long long)xx * cp + c]));
            }
        }
    }
    for (int s = 32; s >= 1; s >>= 1) m = fmaxf(m, __shfl_xor(m, s));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < NT / 64; ++w) m = fmaxf(m, red[w]);
        atomicMax(amax, __float_as_uint(m));
    }
}


// ---------------------------------------------------------------------------------------------------------------------
// elementwise helpers on padded NHWC channel slices
// ---------------------------------------------------------------------------------------------------------------------
__device__ __forceinline__ long long pix_index(long long idx, int C, int B, int H, int W, int *c) {
    *c = idx % C;
    long long q = idx / C;
    const int x = q % W;
    q /= W;
    const int y = q % H;
    const int b = q / H;
    return ((long long)b * (H + 2) + y + 1) * (W + 2) + x + 1;
}

// out = a·x1 + b·x2 on 8-channel groups; an operand in the split-f16 layout holds values scaled by S (gscale_of):
// it is read as (hi + lo) / S, and a split output is written as v·S (overflow flagged like the x3 convs)
__device__ __forceinline__ void ld8(const void *base, long long pix, int cp, int coff, int split, float inv_s,
                                    float v[8]) {
    if (split) {
        const unsigned char *g = static_cast<const unsigned char *>(base) + (pix * cp + coff) * 4;
        const f16x8 h = *reinterpret_cast<const f16x8 *>(g), l = *reinterpret_cast<const f16x8 *>(g + 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ((float)h[e] + (float)l[e]) * inv_s;
    } else {
        const float *f = static_cast<const float *>(base) + pix * cp + coff;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f[e];
    }
}

__global__ void axpby_gs_kernel(void *out, int o_cp, int o_coff, int o_split, float a, const void *x1, int x1_cp,
                                int x1_coff, int x1_split, float b, const void *x2, int x2_cp, int x2_coff,
                                int x2_split, int C, int B, int H, int W, const unsigned *amax, int *overflow) {
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    const int G = C / 8;
    if (idx >= (long long)B * H * W * G) return;
    int g;
    const long long pix = pix_index(idx, G, B, H, W, &g);
    const float S = gscale_of(amax), inv_s = 1.f / S;
    float v[8], w[8];
    ld8(x1, pix, x1_cp, x1_coff + 8 * g, x1_split, inv_s, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= a;
    if (x2) {
        ld8(x2, pix, x2_cp, x2_coff + 8 * g, x2_split, inv_s, w);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += b * w[e];
    }
    if (o_split) {
        f16x8 h, l;
        bool ok = true;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float x = v[e] * S;
            h[e] = (_Float16)x;
            l[e] = (_Float16)(x - (float)h[e]);
            ok = ok && fabsf(x) < 65504.f;
        }
        unsigned char *p = static_cast<unsigned char *>(out) + (pix * o_cp + o_coff + 8 * g) * 4;
        *reinterpret_cast<f16x8 *>(p) = h;
        *reinterpret_cast<f16x8 *>(p + 16) = l;
        if (!ok && overflow) atomicOr(overflow, 1);
    } else {
        float *f = static_cast<float *>(out) + pix * o_cp + o_coff + 8 * g;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = v[e];
    }
}

// axpby_gs_kernel's per-element arithmetic (bitwise the same results) on whole image rows: a block walks rows
// row = blockIdx.x + k·gridDim.x, the index math per row instead of a 64-bit division chain per 8-channel group
// (config-3 step -0.5 ms, profiles/r4_axpby_rows_ab.txt).
__global__ void axpby_rows_kernel(void *out, int o_cp, int o_coff, int o_split, float a, const void *x1, int x1_cp,
                                  int x1_coff, int x1_split, float b, const void *x2, int x2_cp, int x2_coff,
                                  int x2_split, int C, int B, int H, int W, const unsigned *amax, int *overflow) {
    const float S = gscale_of(amax), inv_s = 1.f / S;
    const int G = C / 8;
    bool ok = true;
    for (long long row = blockIdx.x; row < (long long)B * H; row += gridDim.x) {
        const long long bb = row / H, y = row - bb * H;
        const long long pix0 = (bb * (H + 2) + y + 1) * (W + 2) + 1;
        for (int k = threadIdx.x; k < W * G; k += NT) {
            const int xx = k / G, g = k - xx * G;
            const long long pix = pix0 + xx;
            float v[8], w[8];
            ld8(x1, pix, x1_cp, x1_coff + 8 * g, x1_split, inv_s, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= a;
            if (x2) {
                ld8(x2, pix, x2_cp, x2_coff + 8 * g, x2_split, inv_s, w);
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] += b * w[e];
            }
            if (o_split) {
                f16x8 h, l;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float x = v[e] * S;
                    h[e] = (_Float16)x;
                    l[e] = (_Float16)(x - (float)h[e]);
                    ok = ok && fabsf(x) < 65504.f;
                }
                unsigned char *p = static_cast<unsigned char *>(out) + (pix * o_cp + o_coff + 8 * g) * 4;
                *reinterpret_cast<f16x8 *>(p) = h;
                *reinterpret_cast<f16x8 *>(p + 16) = l;
            } else {
                float *f = static_cast<float *>(out) + pix * o_cp + o_coff + 8 * g;
#pragma unroll
                for (int e = 0; e < 8; ++e) f[e] = v[e];
            }
        }
    }
    if (!ok && overflow) atomicOr(overflow, 1);
}

// axpby_rows_kernel with U (pixel, 8-channel group) items per thread in flight: all their loads are issued before any
// arithmetic or store (the one-item loop keeps one load pair per thread in flight: ~2.7 TB/s at config 5).  Bitwise the
// same per-element arithmetic.
template <int U>
__global__ void axpby_rows_u_kernel(void *out, int o_cp, int o_coff, int o_split, float a, const void *x1, int x1_cp,
                                    int x1_coff, int x1_split, float b, const void *x2, int x2_cp, int x2_coff,
                                    int x2_split, int C, int B, int H, int W, const unsigned *amax, int *overflow) {
    const float S = gscale_of(amax), inv_s = 1.f / S;
    const int G = C / 8;
    bool ok = true;
    for (long long row = blockIdx.x; row < (long long)B * H; row += gridDim.x) {
        const long long bb = row / H, y = row - bb * H;
        const long long pix0 = (bb * (H + 2) + y + 1) * (W + 2) + 1;
        for (int k0 = threadIdx.x; k0 < W * G; k0 += U * NT) {
            float v[U][8], w[U][8];
            long long pix[U];
            int g[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = k0 + u * NT;
                const int kk = k < W * G ? k : k0;  // (past the row: a repeat of item k0, not stored)
                const int xx = kk / G;
                g[u] = kk - xx * G;
                pix[u] = pix0 + xx;
                ld8(x1, pix[u], x1_cp, x1_coff + 8 * g[u], x1_split, inv_s, v[u]);
                if (x2) ld8(x2, pix[u], x2_cp, x2_coff + 8 * g[u], x2_split, inv_s, w[u]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (k0 + u * NT >= W * G) break;
#pragma unroll
                for (int e = 0; e < 8; ++e) v[u][e] *= a;
                if (x2) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[u][e] += b * w[u][e];
                }
                if (o_split) {
                    f16x8 h, l;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float x = v[u][e] * S;
                        h[e] = (_Float16)x;
                        l[e] = (_Float16)(x - (float)h[e]);
                        ok = ok && fabsf(x) < 65504.f;
                    }
                    unsigned char *p = static_cast<unsigned char *>(out) + (pix[u] * o_cp + o_coff + 8 * g[u]) * 4;
                    *reinterpret_cast<f16x8 *>(p) = h;
                    *reinterpret_cast<f16x8 *>(p + 16) = l;
                } else {
                    float *f = static_cast<float *>(out) + pix[u] * o_cp + o_coff + 8 * g[u];
#pragma unroll
                    for (int e = 0; e < 8; ++e) f[e] = v[u][e];
                }
            }
        }
    }
    if (!ok && overflow) atomicOr(overflow, 1);
}

// out = a·x1 + b·x2 (fp32 out and x1, x2 split at scale S(amax)) on 64-channel slices, with max |out| OR-ed into
// *out_amax: the closing add of an RRDB's x3 backward, whose result is the next RRDB's gradient-scale source
// (esr_grad_amax fused).  A block walks whole image rows like grad_amax_kernel (16-B loads, index math per row) and
// issues ONE atomic (one per wave, on the same word, cost 4 ms per config-3 step).
__global__ void axpby_amax_kernel(float *out, int o_cp, int o_coff, float a, const float *x1, int x1_cp, int x1_coff,
                                  float b, const void *x2, int x2_cp, int x2_coff, int x2_split, int C, int B, int H,
                                  int W, const unsigned *amax, unsigned *out_amax) {
    __shared__ float red[NT / 64];
    const float inv_s = 1.f / gscale_of(amax);
    const int G = C / 8;
    float mx = 0.f;
    for (long long row = blockIdx.x; row < (long long)B * H; row += gridDim.x) {
        const long long bb = row / H, y = row - bb * H;
        const long long pix0 = (bb * (H + 2) + y + 1) * (W + 2) + 1;
        for (int k = threadIdx.x; k < W * G; k += NT) {
            const int xx = k / G, g = k - xx * G;
            const long long pix = pix0 + xx;
            float v[8], w[8];
            ld8(x1, pix, x1_cp, x1_coff + 8 * g, 0, 1.f, v);
            ld8(x2, pix, x2_cp, x2_coff + 8 * g, x2_split, inv_s, w);
            float *f = out + pix * o_cp + o_coff + 8 * g;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float r = v[e] * a;  // (the expression of axpby_gs_kernel: the same rounding)
                r += b * w[e];
                f[e] = r;
                mx = fmaxf(mx, fabsf(r));
            }
        }
    }
    for (int sh = 32; sh >= 1; sh >>= 1) mx = fmaxf(mx, __shfl_xor(mx, sh));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int wv = 1; wv < NT / 64; ++wv) mx = fmaxf(mx, red[wv]);
        atomicMax(out_amax, __float_as_uint(mx));
    }
}

__global__ void lrelu_bwd_kernel(float *d, int d_cp, int d_coff, const float *y, int y_cp, int y_coff, int C, int B,
                                 int H, int W, int y_split) {
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= (long long)B * H * W * C) return;
    int c;
    const long long pix = pix_index(idx, C, B, H, W, &c);
    const float yv = y_split ? split_at(reinterpret_cast<const unsigned char *>(y) + pix * y_cp * 4, y_coff + c)
                             : y[pix * y_cp + y_coff + c];
    if (!(yv > 0.f)) d[pix * d_cp + d_coff + c] *= 0.2f;
}

// lrelu_bwd_kernel on 8-channel groups (C, offsets and pitches multiples of 8, 16-B aligned; y split or fp32): two
// 16-B loads of d and of y per thread and one index computation per group instead of per element
__global__ void lrelu_bwd8_kernel(float *d, int d_cp, int d_coff, const float *y, int y_cp, int y_coff, int C, int B,
                                  int H, int W, int y_split) {
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    const int G = C / 8;
    if (idx >= (long long)B * H * W * G) return;
    int g;
    const long long pix = pix_index(idx, G, B, H, W, &g);
    float yv[8];
    if (y_split) {
        const unsigned char *q = reinterpret_cast<const unsigned char *>(y) + (pix * y_cp + y_coff + 8 * g) * 4;
        const f16x8 h = *reinterpret_cast<const f16x8 *>(q), l = *reinterpret_cast<const f16x8 *>(q + 16);
#pragma unroll
        for (int e = 0; e < 8; ++e) yv[e] = (float)h[e] + (float)l[e];
    } else {
        const f32x4 a = *reinterpret_cast<const f32x4 *>(y + pix * y_cp + y_coff + 8 * g);
        const f32x4 b = *reinterpret_cast<const f32x4 *>(y + pix * y_cp + y_coff + 8 * g + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { yv[e] = a[e]; yv[e + 4] = b[e]; }
    }
    f32x4 *dp = reinterpret_cast<f32x4 *>(d + pix * d_cp + d_coff + 8 * g);
    f32x4 a = dp[0], b = dp[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (!(yv[e] > 0.f)) a[e] *= 0.2f;
        if (!(yv[e + 4] > 0.f)) b[e] *= 0.2f;
    }
    dp[0] = a;
    dp[1] = b;
}

__global__ void axpby_kernel(float *out, int o_cp, int o_coff, float a, const float *x1, int x1_cp, int x1_coff,
                             float b, const float *x2, int x2_cp, int x2_coff, int C, int B, int H, int W) {
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= (long long)B * H * W * C) return;
    int c;
    const long long pix = pix_index(idx, C, B, H, W, &c);
    float v = a * x1[pix * x1_cp + x1_coff + c];
    if (x2) v += b * x2[pix * x2_cp + x2_coff + c];
    out[pix * o_cp + o_coff + c] = v;
}

// out (grid H×W) = Σ over each 2×2 block of src (grid 2H×2W)
__global__ void sum2x2_kernel(float *out, int o_cp, int o_coff, const float *src, int s_cp, int s_coff, int C, int B,
                              int H, int W) {
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= (long long)B * H * W * C) return;
    const int c = idx % C;
    long long q = idx / C;
    const int x = q % W;
    q /= W;
    const int y = q % H;
    const int b = q / H;
    float v = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int e = 0; e < 2; ++e)
            v += src[(((long long)b * (2 * H + 2) + 2 * y + a + 1) * (2 * W + 2) + 2 * x + e + 1) * s_cp + s_coff + c];
    out[(((long long)b * (H + 2) + y + 1) * (W + 2) + x + 1) * o_cp + o_coff + c] = v;
}

__global__ void nchw_to_padded_kernel(const float *src, int C, int B, int H, int W, float *dst, int d_cp, int d_coff,
                                      int to_nchw) {
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= (long long)B * C * H * W) return;
    const int x = idx % W;
    const int y = (idx / W) % H;
    const int c = (idx / ((long long)W * H)) % C;
    const int b = idx / ((long long)W * H * C);
    const long long pix = ((long long)b * (H + 2) + y + 1) * (W + 2) + x + 1;
    if (to_nchw) const_cast<float *>(src)[idx] = dst[pix * d_cp + d_coff + c];
    else dst[pix * d_cp + d_coff + c] = src[idx];
}

// ---------------------------------------------------------------------------------------------------------------------
// CEM adjoint
// ---------------------------------------------------------------------------------------------------------------------
// (o, u) pairs of one dimension with clamp(s*o + c + u - pd, 0, L-1) == k: for a fixed u, an o-range [lo, hi].
__device__ __forceinline__ bool o_range(int k, int u, int s, int c, int pd, int L, int O, int *lo, int *hi) {
    const int base = c + u - pd;  // position = s*o + base
    int a, b;
    if (k > 0 && k < L - 1) {
        const int t = k - base;
        if (t < 0 || t % s) return false;
        a = b = t / s;
    } else if (k == 0) {  // s*o + base <= 0
        a = 0;
        const int t = -base;
        if (t < 0) return false;
        b = t / s;
        if (L == 1) b = O - 1;
    } else {  // k == L-1: s*o + base >= L-1
        const int t = L - 1 - base;
        a = t <= 0 ? 0 : (t + s - 1) / s;
        b = O - 1;
    }
    if (a < 0) a = 0;
    if (b > O - 1) b = O - 1;
    if (a > b) return false;
    *lo = a;
    *hi = b;
    return true;
}

struct AdjParams {
    const float *g;   // [B*C][Oy][Ox]
    float *out;       // [B*C][Ny][Nx] with Ny = ceil(Ly/os) sampled at k = os*i + oc
    const float *w;   // [K][K] forward taps
    int K, s, c, Ly, Lx, Oy, Ox, os, oc, Ny, Nx, planes;
    float alpha;      // out = alpha * F^T(g) (+ beta * out when accumulate)
    int accumulate;
    int fast;         // interior fast path (default; esr_cem_adjoint flags bit 1 = generic)
};

// The border outputs of the stride-1 adjoint (row or column 0 / L-1, where the replicate clamp lands whole tap rows /
// columns of g): one block per output, the generic per-tap range sums split over the block's threads (tap q = thread
// + 256 k) and added in a fixed tree order.  (One thread per border output ran 16 k threads of ~K²·K/2 serial adds each
// for the 41² inverse filter: ≈5 ms per config-5 iteration.)
__global__ __launch_bounds__(256) void cem_adjoint_border_kernel(AdjParams p) {
    __shared__ float red[256];
    const int nb = 2 * p.Nx + 2 * (p.Ny - 2);
    const long long plane = blockIdx.x / nb;
    const int k = (int)(blockIdx.x - plane * nb);
    int i, j;
    if (k < 2 * p.Nx) {
        i = k < p.Nx ? 0 : p.Ny - 1;
        j = k < p.Nx ? k : k - p.Nx;
    } else {
        i = 1 + (k - 2 * p.Nx) / 2;
        j = ((k - 2 * p.Nx) & 1) ? p.Nx - 1 : 0;
    }
    const int ky = p.os * i + p.oc, kx = p.os * j + p.oc, pd = p.K / 2;
    const float *g = p.g + plane * p.Oy * p.Ox;
    float acc = 0.f;
    for (int q = threadIdx.x; q < p.K * p.K; q += 256) {
        const int uy = q / p.K, ux = q - uy * p.K;
        int ylo, yhi, xlo, xhi;
        if (!o_range(ky, uy, p.s, p.c, pd, p.Ly, p.Oy, &ylo, &yhi)) continue;
        if (!o_range(kx, ux, p.s, p.c, pd, p.Lx, p.Ox, &xlo, &xhi)) continue;
        float sg = 0.f;
        for (int oy = ylo; oy <= yhi; ++oy)
            for (int ox = xlo; ox <= xhi; ++ox) sg += g[(long long)oy * p.Ox + ox];
        acc += p.w[q] * sg;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        float *o = p.out + (plane * p.Ny + i) * p.Nx + j;
        *o = p.accumulate ? *o + p.alpha * red[0] : p.alpha * red[0];
    }
}

// Stride-1 adjoint (the inverse filter's, CEMnet.py:149-151: s = os = 1, oc = 0), interior outputs, tiled as
// cem_inv_tiled: out[k] = Σ_u w[u] · g0[k - c + pd - u] with g0 = g zero-extended, i.e. a correlation of g0 with the
// taps reversed.  A 64 × 16 block of outputs stages its (16 + K - 1) × (64 + K - 1) g0 window in LDS once; each thread
// slides a 4-wide register window along every tap row.  Taps are visited in the generic loop's order (uy, then ux,
// ascending: window rows and columns descending), so interior outputs are bitwise those of cem_adjoint_kernel; border
// outputs (where the replicate clamp adds terms) are left to cem_adjoint_border_kernel.  The per-output loop on the
// inverse filter's 41² taps of the KernelGAN-recipe kernel took 9.6 ms per config-5 iteration.
__global__ __launch_bounds__(256) void cem_adjoint_s1_tiled(AdjParams p) {
    extern __shared__ float smem[];
    const int K = p.K, pd = K / 2, WP = 64 + K - 1, WR = 16 + K - 1;
    float *sw = smem;                           // [WR][WP]
    float *swt = smem + WR * WP;                // the K × K taps (read from LDS: see cem_inv_tiled)
    for (int k = threadIdx.x; k < K * K; k += 256) swt[k] = p.w[k];
    const int j0 = blockIdx.x * 64, i0 = blockIdx.y * 16;
    const long long plane = blockIdx.z;
    const float *g = p.g + plane * p.Oy * p.Ox;
    const int org = -p.c - pd;                  // window origin relative to the output index (k - c + pd - (K - 1))
    for (int y = threadIdx.x / 64; y < WR; y += 4) {
        const int gy = i0 + y + org;
        for (int x = threadIdx.x % 64; x < WP; x += 64) {
            const int gx = j0 + x + org;
            sw[y * WP + x] = (gy >= 0 && gy < p.Oy && gx >= 0 && gx < p.Ox) ? g[(long long)gy * p.Ox + gx] : 0.f;
        }
    }
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int uy = 0; uy < K; ++uy) {
        // window row K-1-uy, columns 4tx + (K-1-ux) (+ e for output e): ux ascending = columns descending
        const float *sr = sw + (ty + K - 1 - uy) * WP + 4 * tx;
        const float *wr = swt + uy * K;  // broadcast LDS reads (not scalar loads: cem_inv_tiled)
        float r1 = sr[K - 1 + 1], r2 = sr[K - 1 + 2], r3 = sr[K - 1 + 3];
        for (int ux = 0; ux < K; ++ux) {
            const int v = K - 1 - ux;
            const float r0 = sr[v], w = wr[ux];
            a0 += w * r0;
            a1 += w * r1;
            a2 += w * r2;
            a3 += w * r3;
            r3 = r2;
            r2 = r1;
            r1 = r0;
        }
    }
    const int i = i0 + ty;
    if (i >= p.Ny || i == 0 || i == p.Ly - 1) return;
    float *o = p.out + (plane * p.Ny + i) * p.Nx;
    const float a[4] = {a0, a1, a2, a3};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int j = j0 + 4 * tx + e;
        if (j >= p.Nx || j == 0 || j == p.Lx - 1) continue;
        o[j] = p.accumulate ? o[j] + p.alpha * a[e] : p.alpha * a[e];
    }
}


__global__ __launch_bounds__(NT) void cem_adjoint_kernel(AdjParams p) {
    __shared__ float sw[64 * 64];
    for (int i = threadIdx.x; i < p.K * p.K; i += NT) sw[i] = p.w[i];
    __syncthreads();
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= (long long)p.planes * p.Ny * p.Nx) return;
    const int j = idx % p.Nx, i = (idx / p.Nx) % p.Ny;
    const long long plane = idx / ((long long)p.Nx * p.Ny);
    const int ky = p.os * i + p.oc, kx = p.os * j + p.oc;
    const float *g = p.g + plane * p.Oy * p.Ox;
    const int pd = p.K / 2;
    float acc = 0.f;
    if (p.fast && ky > 0 && ky < p.Ly - 1 && kx > 0 && kx < p.Lx - 1) {
        // interior (no replicate clamp lands here): only the taps with s | (k - c - u + pd) contribute, one o each.
        // The generic loop below visits the same taps in the same order and adds the same products (its sg is the
        // one g value), so the two are bitwise equal (tests/test_gpu_cem_adjoint.py) — without its per-tap range
        // search over all K² taps.
        const int ty = ky - p.c + pd, tx = kx - p.c + pd;
        const int ry = ((ty % p.s) + p.s) % p.s, rx = ((tx % p.s) + p.s) % p.s;
        for (int uy = ry; uy < p.K; uy += p.s) {
            const int oy = (ty - uy) / p.s;
            if (oy < 0 || oy >= p.Oy) continue;
            const float *gr = g + (long long)oy * p.Ox;
            for (int ux = rx; ux < p.K; ux += p.s) {
                const int ox = (tx - ux) / p.s;
                if (ox < 0 || ox >= p.Ox) continue;
                acc += sw[uy * p.K + ux] * gr[ox];
            }
        }
        float *o = p.out + plane * p.Ny * p.Nx + (long long)i * p.Nx + j;
        *o = p.accumulate ? *o + p.alpha * acc : p.alpha * acc;
        return;
    }
    for (int uy = 0; uy < p.K; ++uy) {
        int ylo, yhi;
        if (!o_range(ky, uy, p.s, p.c, pd, p.Ly, p.Oy, &ylo, &yhi)) continue;
        for (int ux = 0; ux < p.K; ++ux) {
            int xlo, xhi;
            if (!o_range(kx, ux, p.s, p.c, pd, p.Lx, p.Ox, &xlo, &xhi)) continue;
            const float wv = sw[uy * p.K + ux];
            float sg = 0.f;
            for (int oy = ylo; oy <= yhi; ++oy)
                for (int ox = xlo; ox <= xhi; ++ox) sg += g[(long long)oy * p.Ox + ox];
            acc += wv * sg;
        }
    }
    float *o = p.out + plane * p.Ny * p.Nx + (long long)i * p.Nx + j;
    *o = p.accumulate ? *o + p.alpha * acc : p.alpha * acc;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------------------------
// generator input adjoint (Z optimisation): replicate pre-pad adjoint + bilinear ↓sf adjoint
// ---------------------------------------------------------------------------------------------------------------------
// One thread per output PIXEL, all C channels (the HR / LR gradient slots are C consecutive channels of a pixel
// record of hr_cp / lr_cp floats: one sector per pixel instead of one per (pixel, channel) — the per-channel threads
// re-fetched each 288-B HR record three times, 2.4 ms per config-5 iteration).  Same adds in the same order per output.
// The four corner outputs collect a (M+1)² block of the padded grid each (M = 88 at config 5: 7921 positions × C in
// one thread held the launch for 2.3 ms): they are left to input_adjoint_corner_kernel, a block per corner.
struct InAdj {
    const float *d_hr;
    int hr_cp, hr_coff;
    const float *d_lr;
    int lr_cp, lr_coff, sf;
    const float *d_pl;
    int C, B, Hp, Wp, M;
};

// the gradient reaching padded position (yp, xp), channel c, from the HR slot, the planar term and the LR slot
__device__ __forceinline__ float in_adj_term(const InAdj &q, int b, int c, int yp, int xp) {
    float v = 0.f;
    const int Hl = q.sf > 0 ? q.Hp / q.sf : 0, Wl = q.sf > 0 ? q.Wp / q.sf : 0;
    if (q.d_hr) v += q.d_hr[(((long long)b * (q.Hp + 2) + yp + 1) * (q.Wp + 2) + xp + 1) * q.hr_cp + q.hr_coff + c];
    if (q.d_pl) v += q.d_pl[(((long long)b * q.C + c) * q.Hp + yp) * q.Wp + xp];
    if (q.d_lr) {  // bilinear ↓sf, align_corners=False: sf = 4: mean of the central 2×2 of each 4×4 block; sf = 2: of the 2×2 block
        const int ry = yp % q.sf, rx = xp % q.sf;
        if ((ry == q.sf / 2 - 1 || ry == q.sf / 2) && (rx == q.sf / 2 - 1 || rx == q.sf / 2))
            v += 0.25f * q.d_lr[(((long long)b * (Hl + 2) + yp / q.sf + 1) * (Wl + 2) + xp / q.sf + 1) * q.lr_cp +
                                q.lr_coff + c];
    }
    return v;
}

__global__ void input_adjoint_kernel(InAdj q, float *out) {
    const int Ho = q.Hp - 2 * q.M, Wo = q.Wp - 2 * q.M;
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= (long long)q.B * Ho * Wo) return;
    const int X = idx % Wo;
    const int Y = (idx / Wo) % Ho;
    const int b = idx / ((long long)Wo * Ho);
    if (q.M > 0 && (Y == 0 || Y == Ho - 1) && (X == 0 || X == Wo - 1)) return;  // a corner: the corner kernel
    // padded positions that the replicate pad clamps onto (Y, X)
    const int y0 = Y == 0 ? 0 : Y + q.M, y1 = Y == Ho - 1 ? q.Hp - 1 : Y + q.M;
    const int x0 = X == 0 ? 0 : X + q.M, x1 = X == Wo - 1 ? q.Wp - 1 : X + q.M;
    for (int c = 0; c < q.C; ++c) {
        float v = 0.f;
        for (int yp = y0; yp <= y1; ++yp)
            for (int xp = x0; xp <= x1; ++xp) {
                if (q.d_hr) v += q.d_hr[(((long long)b * (q.Hp + 2) + yp + 1) * (q.Wp + 2) + xp + 1) * q.hr_cp +
                                        q.hr_coff + c];
                if (q.d_pl) v += q.d_pl[(((long long)b * q.C + c) * q.Hp + yp) * q.Wp + xp];
                if (q.d_lr) {
                    const int Hl = q.Hp / q.sf, Wl = q.Wp / q.sf;
                    const int ry = yp % q.sf, rx = xp % q.sf;
                    if ((ry == q.sf / 2 - 1 || ry == q.sf / 2) && (rx == q.sf / 2 - 1 || rx == q.sf / 2))
                        v += 0.25f * q.d_lr[(((long long)b * (Hl + 2) + yp / q.sf + 1) * (Wl + 2) + xp / q.sf + 1) *
                                                q.lr_cp + q.lr_coff + c];
                }
            }
        out[(((long long)b * q.C + c) * Ho + Y) * Wo + X] = v;
    }
}

// block (b, corner k): the (M+1)² padded positions of that corner, per channel: each thread sums its strided share
// of the positions (whole terms, in position order), then the 256 thread sums are added in thread order
__global__ void input_adjoint_corner_kernel(InAdj q, float *out) {
    __shared__ float red[NT];
    const int Ho = q.Hp - 2 * q.M, Wo = q.Wp - 2 * q.M;
    const int b = blockIdx.x >> 2, k = blockIdx.x & 3;
    const int Y = (k & 2) ? Ho - 1 : 0, X = (k & 1) ? Wo - 1 : 0;
    const int y0 = Y == 0 ? 0 : Y + q.M, y1 = Y == Ho - 1 ? q.Hp - 1 : Y + q.M;
    const int x0 = X == 0 ? 0 : X + q.M, x1 = X == Wo - 1 ? q.Wp - 1 : X + q.M;
    const int nx = x1 - x0 + 1, n = (y1 - y0 + 1) * nx;
    for (int c = 0; c < q.C; ++c) {
        float v = 0.f;
        for (int e = threadIdx.x; e < n; e += NT) v += in_adj_term(q, b, c, y0 + e / nx, x0 + e % nx);
        red[threadIdx.x] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            float t = 0.f;
            for (int r = 0; r < NT; ++r) t += red[r];
            out[(((long long)b * q.C + c) * Ho + Y) * Wo + X] = t;
        }
        __syncthreads();
    }
}

extern "C" int esr_conv3x3_wgrad(const float *in, int32_t in_cp, int32_t cin, int32_t flags, const float *dout,
                                 int32_t dout_cp, int32_t dout_coff, int32_t cout, int32_t B, int32_t H, int32_t W,
                                 int32_t splits, float *partial, esr_stream_t stream) {
    const int up2 = flags & 1, split = (flags >> 1) & 1, x3 = (flags >> 2) & 1, dsplit = (flags >> 3) & 1;
    if (!in || !dout || !partial || cin <= 0 || cin % 4 || in_cp % 4 || cout <= 0 || cout > 64 || B <= 0 ||
        H <= 0 || W <= 0 || splits <= 0 || (up2 && (H % 2 || W % 2)) || (flags & ~15) ||
        (split && (cin % 8 || in_cp % 8 || (!x3 && g_wgrad_kernel != 1))) || (x3 && !split) ||
        (dsplit && (!x3 || cout % 8 || dout_cp % 8 || dout_coff % 8)))
        return ESR_EINVAL;
    WgradParams p;
    p.in = in; p.in_cp = in_cp; p.cin = cin; p.up2 = up2;
    p.dout = dout; p.dout_cp = dout_cp; p.dout_coff = dout_coff; p.cout = cout; p.cout_pad = cout > 32 ? 64 : 32;
    p.B = B; p.H = H; p.W = W;
    p.tiles_x = (W + WT_TW - 1) / WT_TW; p.tiles_y = (H + WT_TH - 1) / WT_TH;
    p.splits = splits; p.cin_pad = (cin + 31) / 32 * 32;
    p.partial = partial;
    p.dsplit = dsplit;
    p.dbg = g_wgrad3d_dbg;
    const unsigned total = (unsigned)(p.cin_pad / 32 * splits);
    if (x3 && dsplit && g_wgrad3_dma) {
        const unsigned grid = 8 * ((total + 7) / 8);
        const hipStream_t st = (hipStream_t)stream;
        if (p.cout_pad == 64) {
            p.tiles_y = (H + 3) / 4;
#ifdef ESR_X3_EXPERIMENTS
            if (g_wgrad3d_unroll == 1)
                hipLaunchKernelGGL((wgrad3d_kernel<2, 4, 1>), dim3(grid), dim3(W3D<2, 4>::NT), 0, st, p);
            else if (g_wgrad3d_unroll == 2)
                hipLaunchKernelGGL((wgrad3d_kernel<2, 4, 2>), dim3(grid), dim3(W3D<2, 4>::NT), 0, st, p);
            else
#endif
            hipLaunchKernelGGL((wgrad3d_kernel<2, 4>), dim3(grid), dim3(W3D<2, 4>::NT), 0, st, p);
        } else {
#ifdef ESR_X3_EXPERIMENTS
            if (g_wgrad3d_unroll == 1)
                hipLaunchKernelGGL((wgrad3d_kernel<1, 8, 1>), dim3(grid), dim3(W3D<1, 8>::NT), 0, st, p);
            else if (g_wgrad3d_unroll == 2)
                hipLaunchKernelGGL((wgrad3d_kernel<1, 8, 2>), dim3(grid), dim3(W3D<1, 8>::NT), 0, st, p);
            else
#endif
            hipLaunchKernelGGL((wgrad3d_kernel<1, 8>), dim3(grid), dim3(W3D<1, 8>::NT), 0, st, p);
        }
    } else if (x3) {
        const unsigned grid = 8 * ((total + 7) / 8);
        const hipStream_t st = (hipStream_t)stream;
        if (p.cout_pad == 64)
            hipLaunchKernelGGL((wgrad3_kernel<2>), dim3(grid), dim3(W3<2>::NT), 0, st, p);
        else
            hipLaunchKernelGGL((wgrad3_kernel<1>), dim3(grid), dim3(W3<1>::NT), 0, st, p);
    } else if (g_wgrad_kernel == 1) {
        const unsigned grid = 8 * ((total + 7) / 8);  // whole XCD rounds; the surplus workgroups exit at once
        const hipStream_t st = (hipStream_t)stream;
        if (split) {
            if (p.cout_pad == 64)
                hipLaunchKernelGGL((wgrad2_kernel<2, true>), dim3(grid), dim3(W2<2>::NT), 0, st, p);
            else
                hipLaunchKernelGGL((wgrad2_kernel<1, true>), dim3(grid), dim3(W2<1>::NT), 0, st, p);
        } else {
            if (p.cout_pad == 64)
                hipLaunchKernelGGL((wgrad2_kernel<2, false>), dim3(grid), dim3(W2<2>::NT), 0, st, p);
            else
                hipLaunchKernelGGL((wgrad2_kernel<1, false>), dim3(grid), dim3(W2<1>::NT), 0, st, p);
        }
    } else {
        hipLaunchKernelGGL(wgrad_kernel, dim3(total), dim3(256), 0, (hipStream_t)stream, p);
    }
    return launched();
}

extern "C" int esr_wgrad_reduce(const float *partial, int32_t splits, int64_t n, float scale, float *out,
                                esr_stream_t stream) {
    if (!partial || !out || splits <= 0 || n <= 0) return ESR_EINVAL;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + RED_O - 1) / RED_O)), dim3(NT), 0,
                       (hipStream_t)stream, partial, splits, n, scale, out, nullptr);
    return launched();
}

extern "C" int esr_wgrad_reduce_gs(const float *partial, int32_t splits, int64_t n, float scale, const uint32_t *amax,
                                   float *out, esr_stream_t stream) {
    if (!partial || !out || !amax || splits <= 0 || n <= 0) return ESR_EINVAL;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + RED_O - 1) / RED_O)), dim3(NT), 0,
                       (hipStream_t)stream, partial, splits, n, scale, out, amax);
    return launched();
}

extern "C" int esr_wgrad_reduce2(const float *partial, int32_t splits, int64_t n, int64_t n_w, float scale_w,
                                 float scale_b, const uint32_t *amax, float *out, esr_stream_t stream) {
    if (!partial || !out || splits <= 0 || n <= 0 || n_w < 0 || n_w > n) return ESR_EINVAL;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + RED_O - 1) / RED_O)), dim3(NT), 0,
                       (hipStream_t)stream, partial, splits, n, scale_w, out, amax, (long long)n_w, scale_b);
    return launched();
}

extern "C" int esr_grad_amax(const float *x, int32_t cp, int32_t coff, int32_t C, int32_t B, int32_t H, int32_t W,
                             uint32_t *amax, esr_stream_t stream) {
    if (!x || !amax || C <= 0 || B <= 0 || H <= 0 || W <= 0 || coff + C > cp) return ESR_EINVAL;
    const long long rows = (long long)B * H;
    const unsigned grid = (unsigned)(rows < 2048 ? rows : 2048);
    hipLaunchKernelGGL(grad_amax_kernel, dim3(grid), dim3(NT), 0, (hipStream_t)stream, x, cp, coff, C, B, H, W, amax);
    return launched();
}

extern "C" int esr_axpby_gs(void *out, int32_t o_cp, int32_t o_coff, int32_t o_split, float a, const void *x1,
                            int32_t x1_cp, int32_t x1_coff, int32_t x1_split, float b, const void *x2, int32_t x2_cp,
                            int32_t x2_coff, int32_t x2_split, int32_t C, int32_t B, int32_t H, int32_t W,
                            const uint32_t *amax, int32_t *overflow, esr_stream_t stream) {
    if (!out || !x1 || !amax || C <= 0 || C % 8 || B <= 0 || H <= 0 || W <= 0 || (o_cp | o_coff) % 8 ||
        (x1_cp | x1_coff) % 8 || (x2 && (x2_cp | x2_coff) % 8))
        return ESR_EINVAL;
    const long long rows = (long long)B * H;
    if (g_axpby_rows == 2)
        hipLaunchKernelGGL((axpby_rows_u_kernel<4>), dim3((unsigned)(rows < 2048 ? rows : 2048)), dim3(NT), 0,
                           (hipStream_t)stream, out, o_cp, o_coff, o_split, a, x1, x1_cp, x1_coff, x1_split, b, x2,
                           x2_cp, x2_coff, x2_split, C, B, H, W, amax, overflow);
    else if (g_axpby_rows)
        hipLaunchKernelGGL(axpby_rows_kernel, dim3((unsigned)(rows < 2048 ? rows : 2048)), dim3(NT), 0,
                           (hipStream_t)stream, out, o_cp, o_coff, o_split, a, x1, x1_cp, x1_coff, x1_split, b, x2,
                           x2_cp, x2_coff, x2_split, C, B, H, W, amax, overflow);
    else
        hipLaunchKernelGGL(axpby_gs_kernel, dim3(nblocks((long long)B * H * W * (C / 8))), dim3(NT), 0,
                           (hipStream_t)stream, out, o_cp, o_coff, o_split, a, x1, x1_cp, x1_coff, x1_split, b, x2,
                           x2_cp, x2_coff, x2_split, C, B, H, W, amax, overflow);
    return launched();
}

extern "C" int esr_axpby_gs_amax(float *out, int32_t o_cp, int32_t o_coff, float a, const void *x1, int32_t x1_cp,
                                 int32_t x1_coff, int32_t x1_split, float b, const void *x2, int32_t x2_cp,
                                 int32_t x2_coff, int32_t x2_split, int32_t C, int32_t B, int32_t H, int32_t W,
                                 const uint32_t *amax, uint32_t *out_amax, esr_stream_t stream) {
    if (!out || !x1 || !amax || !out_amax || C <= 0 || C % 8 || B <= 0 || H <= 0 || W <= 0 || (o_cp | o_coff) % 8 ||
        (x1_cp | x1_coff) % 8 || (x2 && (x2_cp | x2_coff) % 8))
        return ESR_EINVAL;
    if (x1_split || !x2) return ESR_EINVAL;  // (the one form the x3 backward uses: fp32 x1, split or fp32 x2)
    const long long rows = (long long)B * H;
    hipLaunchKernelGGL(axpby_amax_kernel, dim3((unsigned)(rows < 2048 ? rows : 2048)), dim3(NT), 0,
                       (hipStream_t)stream, out, o_cp, o_coff, a, static_cast<const float *>(x1), x1_cp, x1_coff, b,
                       x2, x2_cp, x2_coff, x2_split, C, B, H, W, amax, out_amax);
    return launched();
}

static int lrelu_bwd_launch(float *d, int d_cp, int d_coff, const float *y, int y_cp, int y_coff, int C, int B, int H,
                            int W, int y_split, hipStream_t st) {
    const bool g8 = C % 8 == 0 && d_cp % 8 == 0 && d_coff % 8 == 0 && y_cp % 8 == 0 && y_coff % 8 == 0 &&
                    ((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(y)) & 15) == 0;
    if (g8)
        hipLaunchKernelGGL(lrelu_bwd8_kernel, dim3(nblocks((long long)B * H * W * (C / 8))), dim3(NT), 0, st, d, d_cp,
                           d_coff, y, y_cp, y_coff, C, B, H, W, y_split);
    else
        hipLaunchKernelGGL(lrelu_bwd_kernel, dim3(nblocks((long long)B * H * W * C)), dim3(NT), 0, st, d, d_cp, d_coff,
                           y, y_cp, y_coff, C, B, H, W, y_split);
    return launched();
}

extern "C" int esr_lrelu_bwd(float *d, int32_t d_cp, int32_t d_coff, const float *y, int32_t y_cp, int32_t y_coff,
                             int32_t C, int32_t B, int32_t H, int32_t W, esr_stream_t stream) {
    if (!d || !y || C <= 0 || B <= 0 || H <= 0 || W <= 0) return ESR_EINVAL;
    return lrelu_bwd_launch(d, d_cp, d_coff, y, y_cp, y_coff, C, B, H, W, 0, (hipStream_t)stream);
}

extern "C" int esr_lrelu_bwd_split(float *d, int32_t d_cp, int32_t d_coff, const void *y, int32_t y_cp,
                                   int32_t y_coff, int32_t C, int32_t B, int32_t H, int32_t W, esr_stream_t stream) {
    if (!d || !y || C <= 0 || B <= 0 || H <= 0 || W <= 0 || y_cp % 8) return ESR_EINVAL;
    return lrelu_bwd_launch(d, d_cp, d_coff, static_cast<const float *>(y), y_cp, y_coff, C, B, H, W, 1,
                            (hipStream_t)stream);
}

extern "C" int esr_axpby(float *out, int32_t o_cp, int32_t o_coff, float a, const float *x1, int32_t x1_cp,
                         int32_t x1_coff, float b, const float *x2, int32_t x2_cp, int32_t x2_coff, int32_t C,
                         int32_t B, int32_t H, int32_t W, esr_stream_t stream) {
    if (!out || !x1 || C <= 0 || B <= 0 || H <= 0 || W <= 0) return ESR_EINVAL;
    hipLaunchKernelGGL(axpby_kernel, dim3(nblocks((long long)B * H * W * C)), dim3(NT), 0, (hipStream_t)stream, out,
                       o_cp, o_coff, a, x1, x1_cp, x1_coff, b, x2, x2_cp, x2_coff, C, B, H, W);
    return launched();
}

extern "C" int esr_sum2x2(float *out, int32_t o_cp, int32_t o_coff, const float *src, int32_t s_cp, int32_t s_coff,
                          int32_t C, int32_t B, int32_t H, int32_t W, esr_stream_t stream) {
    if (!out || !src || C <= 0 || B <= 0 || H <= 0 || W <= 0) return ESR_EINVAL;
    hipLaunchKernelGGL(sum2x2_kernel, dim3(nblocks((long long)B * H * W * C)), dim3(NT), 0, (hipStream_t)stream, out,
                       o_cp, o_coff, src, s_cp, s_coff, C, B, H, W);
    return launched();
}

extern "C" int esr_nchw_to_padded(const float *src, int32_t C, int32_t B, int32_t H, int32_t W, float *dst,
                                  int32_t d_cp, int32_t d_coff, int32_t to_nchw, esr_stream_t stream) {
    if (!src || !dst || C <= 0 || B <= 0 || H <= 0 || W <= 0 || d_coff + C > d_cp) return ESR_EINVAL;
    hipLaunchKernelGGL(nchw_to_padded_kernel, dim3(nblocks((long long)B * C * H * W)), dim3(NT), 0,
                       (hipStream_t)stream, src, C, B, H, W, dst, d_cp, d_coff, to_nchw);
    return launched();
}

extern "C" int esr_cem_adjoint(const float *g, int32_t planes, int32_t Oy, int32_t Ox, const float *w, int32_t K,
                               int32_t s, int32_t c, int32_t Ly, int32_t Lx, int32_t os, int32_t oc, float alpha,
                               int32_t flags, float *out, esr_stream_t stream) {
    if (!g || !w || !out || planes <= 0 || Oy <= 0 || Ox <= 0 || K <= 0 || K > 64 || !(K & 1) || s <= 0 ||
        Ly <= 0 || Lx <= 0 || os <= 0 || oc < 0 || oc >= os || (flags & ~3))
        return ESR_EINVAL;
    AdjParams p;
    p.g = g; p.out = out; p.w = w; p.K = K; p.s = s; p.c = c; p.Ly = Ly; p.Lx = Lx; p.Oy = Oy; p.Ox = Ox;
    p.os = os; p.oc = oc; p.Ny = (Ly - oc + os - 1) / os; p.Nx = (Lx - oc + os - 1) / os; p.planes = planes;
    p.alpha = alpha; p.accumulate = flags & 1; p.fast = !(flags & 2);
    if (p.fast && s == 1 && os == 1 && oc == 0 && Ly >= 3 && Lx >= 3) {  // the inverse filter's adjoint: tiled
        const size_t lds = ((size_t)(16 + K - 1) * (64 + K - 1) + (size_t)K * K) * sizeof(float);
        hipLaunchKernelGGL(cem_adjoint_s1_tiled, dim3((p.Nx + 63) / 64, (p.Ny + 15) / 16, planes), dim3(256), lds,
                           (hipStream_t)stream, p);
        hipLaunchKernelGGL(cem_adjoint_border_kernel, dim3((unsigned)((long long)planes * (2 * p.Nx + 2 * (p.Ny - 2)))),
                           dim3(256), 0, (hipStream_t)stream, p);
        return launched();
    }
    hipLaunchKernelGGL(cem_adjoint_kernel, dim3(nblocks((long long)planes * p.Ny * p.Nx)), dim3(NT), 0,
                       (hipStream_t)stream, p);
    return launched();
}

extern "C" int esr_input_adjoint(const float *d_hr, int32_t hr_cp, int32_t hr_coff, const float *d_lr, int32_t lr_cp,
                                 int32_t lr_coff, int32_t sf, const float *d_pl, int32_t C, int32_t B, int32_t Hp,
                                 int32_t Wp, int32_t M, float *out, esr_stream_t stream) {
    if (!out || C <= 0 || B <= 0 || M < 0 || Hp - 2 * M <= 0 || Wp - 2 * M <= 0) return ESR_EINVAL;
    if (d_hr && hr_coff + C > hr_cp) return ESR_EINVAL;
    if (d_lr && ((sf != 4 && sf != 2) || Hp % sf || Wp % sf || lr_coff + C > lr_cp)) return ESR_EINVAL;
    const long long n = (long long)B * (Hp - 2 * M) * (Wp - 2 * M);
    const InAdj q{d_hr, hr_cp, hr_coff, d_lr, lr_cp, lr_coff, sf, d_pl, C, B, Hp, Wp, M};
    hipLaunchKernelGGL(input_adjoint_kernel, dim3(nblocks(n)), dim3(NT), 0, (hipStream_t)stream, q, out);
    if (M > 0)
        hipLaunchKernelGGL(input_adjoint_corner_kernel, dim3(4 * B), dim3(NT), 0, (hipStream_t)stream, q, out);
    return launched();
}
