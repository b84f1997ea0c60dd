// esr_conv_x3.hip — 3×3 convolution / polyphase upconv on f16 matrix cores with fp32-level accuracy ("x3" path).
//
// Numerics.  Every fp32 value v is carried as an f16 pair (hi = f16(v), lo = f16(v - hi)), |v - hi - lo| <= 2^-22 |v|
// (absolute 2^-25 below the f16 normal range).  A product a·b is evaluated as a_hi·b_hi + a_hi·b_lo + a_lo·b_hi on
// v_mfma_f32_32x32x16_f16 with fp32 accumulation; the dropped a_lo·b_lo term is <= 2^-22 |ab|.  Three f16 MFMAs
// (3 × 32 cycles per 32×32×16 block) replace eight f32 MFMAs (8 × 64 cycles): 5.3× the MFMA throughput of the
// exact-fp32 path (esr_conv.hip) at ~1e-6 relative error.
//
// Layouts.  Split activations (include/esr_amd.h): per pixel, channels in groups of 8, each group 32 bytes =
// 8 × f16 hi then 8 × f16 lo — 4 bytes per channel like fp32, written once by the producer's epilogue.  Weights:
// packed [chunk16][tap][n_pad][2 groups × 32 B] (64 B per (tap, n)), pre-scaled by a power of two (w_scale) so their lo
// parts stay normal; the epilogue multiplies by 1/w_scale (exact).
//
// Tiling.  The batch is treated as one tall padded image of B·(H+2) rows (the zero halo rows between images are the
// vertical zero padding), so a tile may straddle two images and no per-image row remainder is wasted; output rows that
// fall on halo rows are computed and dropped (2 of H+2).  Tiles are 16 rows × 32 columns, plus one remainder column
// tile of width W % 32 whose 32-pixel M-tiles run row-major across its rows (W = 148 -> 4 full + one 20-wide tile,
// instead of padding to 160).  Workgroup = 512 threads (8 waves, 2 per SIMD); wave w owns M-tiles 2w, 2w+1 × NT
// 32-channel N-tiles.
//
// Pipeline.  K is walked in 16-channel chunks (one 32×32×16 MFMA step per tap).  Each chunk's halo tile (18 × 34
// records of 64 B) and weights are copied HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no
// ds_write) into one of two LDS stages while the MFMAs consume the other stage.  Records are 64 B (4 × 16-B slots)
// with the slot index XOR-swizzled by (record>>2)&3, applied on the DMA source address (the DMA destination is
// lane-linear), so the 16 lanes of every ds_read_b128 group hit 16 distinct slots.  Out-of-range halo pixels and
// the channels past cin of a partial chunk are fetched from a zero page.
// Epilogue: accumulators are re-staged through LDS as fp32 [pixel][channel]; each thread finishes 8-channel groups:
// 1/w_scale, bias, LeakyReLU, residuals (split inputs), split + 16-byte stores, or fp32 planar stores for CEM.
#include <hip/hip_runtime.h>
#include "esr_amd.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glob_void;

constexpr int TH = 16, TWF = 32;
constexpr int HY = TH + 2, HXF = TWF + 2;
constexpr int REC = 64;                            // bytes per staged record (16 channels, split)
constexpr int IN_RECS = (HY * HXF + 15) / 16 * 16;  // 624: whole 16-record DMA wave-instructions
constexpr int NTHR = 512;
constexpr int NWAVES = NTHR / 64;

__device__ __attribute__((aligned(16))) unsigned char g_zero_page[64];

struct X3Params {
    const unsigned char *in;
    int B, H, W, in_cp, cin;
    const unsigned char *w;
    const float *bias;
    float w_scale_inv;
    int cout;
    int tap_y0, tap_x0, tiles_x, tiles_y;
    int *overflow;
    esr_conv_out o;
};

__device__ __forceinline__ float lrelu(float v) { return v > 0.f ? v : 0.2f * v; }

__device__ __forceinline__ void load_group(const unsigned char *p, float v[8]) {
    const f16x8 hi = *reinterpret_cast<const f16x8 *>(p);
    const f16x8 lo = *reinterpret_cast<const f16x8 *>(p + 16);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)hi[j] + (float)lo[j];
}

__device__ __forceinline__ bool store_group(unsigned char *p, const float v[8]) {
    f16x8 hi, lo;
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        hi[j] = (_Float16)v[j];
        lo[j] = (_Float16)(v[j] - (float)hi[j]);
        ok = ok && (fabsf(v[j]) < 65504.f);
    }
    *reinterpret_cast<f16x8 *>(p) = hi;
    *reinterpret_cast<f16x8 *>(p + 16) = lo;
    return ok;
}

// byte offset of logical 16-B slot s of record r inside a stage region
__device__ __forceinline__ int slot_off(int r, int s) { return r * REC + ((s ^ ((r >> 2) & 3)) << 4); }

template <int NT, int TS, int MODE>
__global__ __launch_bounds__(NTHR, 1) void conv_x3_v5(X3Params p) {
    constexpr int T = TS * TS;
    constexpr int N = NT * 32;
    constexpr int W_RECS = T * N;
    constexpr int IN_B = IN_RECS * REC;
    constexpr int W_B = W_RECS * REC;
    constexpr int EP_P = N + 4;
    constexpr int EP_BYTES = TH * TWF * EP_P * 4;
    constexpr int LDS_BYTES = 2 * (IN_B + W_B) > EP_BYTES ? 2 * (IN_B + W_B) : EP_BYTES;
    constexpr int KIN = (IN_RECS / 16 + NWAVES - 1) / NWAVES;
    constexpr int KW = (W_RECS / 16 + NWAVES - 1) / NWAVES;
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int hl = lane >> 5;
    const int ml = lane & 31;

    const int tx = blockIdx.x % p.tiles_x;
    const int ty = blockIdx.x / p.tiles_x;
    const int x0 = tx * TWF;
    const int tw = min(TWF, p.W - x0);
    const int hx = tw + 2;
    const int r0 = ty * TH;
    const int rows_tot = p.B * (p.H + 2);
    const int nq = TH * tw;
    const int nmt = (nq + 31) >> 5;
    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;
    const int nchunk = (p.cin + 15) >> 4;

    const int sub = lane >> 2, ps = lane & 3;
    long long in_src[KIN];
    int in_hi[KIN];
#pragma unroll
    for (int i = 0; i < KIN; ++i) {
        const int k = wave + NWAVES * i;
        const int r = 16 * k + sub;
        const int s = ps ^ ((r >> 2) & 3);
        const int hy = r / hx, hxi = r - (r / hx) * hx;
        const int gy = r0 + hy, gx = x0 + hxi;
        in_hi[i] = -1;
        in_src[i] = 0;
        if (k < IN_RECS / 16 && r < HY * hx && gy < rows_tot && gx < p.W + 2) {
            in_src[i] = (gy * rowp + gx) * pixb + (s << 4);
            in_hi[i] = s >> 1;
        }
    }
    auto dma = [&](int j, int st) {
        const int groups = min(16, p.cin - 16 * j) >> 3;
#pragma unroll
        for (int i = 0; i < KIN; ++i) {
            const int k = wave + NWAVES * i;
            if (k >= IN_RECS / 16) break;
            const void *src = (in_hi[i] >= 0 && in_hi[i] < groups) ? (const void *)(p.in + in_src[i] + 64LL * j)
                                                                   : (const void *)g_zero_page;
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(lds + st * IN_B + k * 1024), 16, 0, 0);
        }
        const unsigned char *wj = p.w + (long long)j * W_B;
#pragma unroll
        for (int i = 0; i < KW; ++i) {
            const int k = wave + NWAVES * i;
            if (k >= W_RECS / 16) break;
            const int r = 16 * k + sub;
            const int s = ps ^ ((r >> 2) & 3);
            __builtin_amdgcn_global_load_lds((glob_void *)(wj + r * REC + (s << 4)),
                                             (lds_void *)(lds + 2 * IN_B + st * W_B + k * 1024), 16, 0, 0);
        }
    };

    int aoff[T][2][2];
    bool mvalid[2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        const int jm = 2 * wave + mt;
        mvalid[mt] = jm < nmt;
        int q = 32 * jm + ml;
        if (q >= nq) q = 0;
        const int rec0 = (q / tw) * hx + q % tw;
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int r = rec0 + (p.tap_y0 + tap / TS) * hx + p.tap_x0 + tap % TS;
            aoff[tap][mt][0] = slot_off(r, 2 * hl);
            aoff[tap][mt][1] = slot_off(r, 2 * hl + 1);
        }
    }
    const int bsw = (ml >> 2) & 3;
    const int boff0 = ml * REC + (((2 * hl) ^ bsw) << 4), boff1 = ml * REC + (((2 * hl + 1) ^ bsw) << 4);

    f32x16 acc[2][NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

    auto compute = [&](const unsigned char *s_in, const unsigned char *s_w) {
        f16x8 ah[2][2], al[2][2], bh[2][NT], bl[2][NT];
        auto ld = [&](int tap, int buf) {
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                ah[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + aoff[tap][mt][0]);
                al[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + aoff[tap][mt][1]);
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                bh[buf][nt] = *reinterpret_cast<const f16x8 *>(s_w + (tap * N + nt * 32) * REC + boff0);
                bl[buf][nt] = *reinterpret_cast<const f16x8 *>(s_w + (tap * N + nt * 32) * REC + boff1);
            }
        };
        ld(0, 0);
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int cb = tap & 1;
            if (tap + 1 < T) ld(tap + 1, cb ^ 1);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[cb][mt], bh[cb][nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bl[cb][nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bh[cb][nt], acc[mt][nt], 0, 0, 0);
        }
    };

    dma(0, 0);
    for (int j = 0; j < nchunk; j += 2) {
        __syncthreads();
        if (j + 1 < nchunk && MODE != 1) dma(j + 1, 1);
        if (mvalid[0]) compute(lds, lds + 2 * IN_B);
        if (j + 1 >= nchunk) break;
        __syncthreads();
        if (j + 2 < nchunk && MODE != 1) dma(j + 2, 0);
        if (mvalid[0]) compute(lds + IN_B, lds + 2 * IN_B + W_B);
    }

    // ---- epilogue: restage fp32 accumulators as [pixel][channel] ----
    __syncthreads();
    float *s_ep = reinterpret_cast<float *>(lds);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        if (!mvalid[mt]) continue;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int q = 32 * (2 * wave + mt) + (r & 3) + 8 * (r >> 2) + 4 * hl;
                if (q < nq) s_ep[q * EP_P + nt * 32 + ml] = acc[mt][nt][r];
            }
    }
    __syncthreads();

    const esr_conv_out &o = p.o;
    const long long orow = (long long)(o.out_w + 2);
    constexpr int GROUPS = N / 8;
    bool ok = true;
    for (int u = tid; u < nq * GROUPS; u += NTHR) {
        const int q = u / GROUPS, g = u - (u / GROUPS) * GROUPS;
        const int c = 8 * g;
        if (c >= p.cout) continue;
        const int R = r0 + 1 + q / tw;  // tall padded row of this output pixel
        const int b = R / (p.H + 2);
        const int y = R - b * (p.H + 2) - 1;
        if (b >= p.B || y < 0 || y >= p.H) continue;
        const int x = x0 + q % tw;
        const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
        const long long opix = ((long long)b * (o.out_h + 2) + oy + 1) * orow + ox + 1;
        float v[8];
        const f32x4 v0 = *reinterpret_cast<const f32x4 *>(s_ep + q * EP_P + c);
        const f32x4 v1 = *reinterpret_cast<const f32x4 *>(s_ep + q * EP_P + c + 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) { v[k] = v0[k]; v[k + 4] = v1[k]; }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float bk = (c + k < p.cout) ? p.bias[c + k] : 0.f;
            v[k] = v[k] * p.w_scale_inv + bk;
            if (o.lrelu) v[k] = lrelu(v[k]);
        }
        if (o.r1) {
            float r[8];
            load_group(reinterpret_cast<const unsigned char *>(o.r1) + (opix * o.r1_cp + o.r1_coff + c) * 4, r);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = o.s1 * v[k] + r[k];
        }
        if (o.r2) {
            float r[8];
            load_group(reinterpret_cast<const unsigned char *>(o.r2) + (opix * o.r2_cp + o.r2_coff + c) * 4, r);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = o.s2 * v[k] + r[k];
        }
        if (o.out_planar) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (c + k < p.cout) o.out[(((long long)b * p.cout + c + k) * o.out_h + oy) * o.out_w + ox] = v[k];
        } else {
            ok &= store_group(reinterpret_cast<unsigned char *>(o.out) + (opix * o.out_cp + o.out_coff + c) * 4, v);
            if (o.out2)
                store_group(reinterpret_cast<unsigned char *>(o.out2) + (opix * o.out2_cp + o.out2_coff + c) * 4, v);
        }
    }
    if (!ok && p.overflow && MODE != 1) atomicOr(p.overflow, 1);
}

}  // namespace

extern "C" int x3exp_conv(int mode, const void *in, int B, int H, int W, int in_cp, int cin, const void *w,
                          const float *bias, float w_scale, int cout, const esr_conv_out *o, int *overflow,
                          void *stream) {
    X3Params p;
    p.in = static_cast<const unsigned char *>(in);
    p.B = B; p.H = H; p.W = W; p.in_cp = in_cp; p.cin = cin;
    p.w = static_cast<const unsigned char *>(w);
    p.bias = bias; p.w_scale_inv = 1.f / w_scale; p.cout = cout;
    p.tap_y0 = 0; p.tap_x0 = 0;
    p.tiles_x = (W + TWF - 1) / TWF;
    p.tiles_y = (B * (H + 2) - 2 + TH - 1) / TH;
    p.overflow = overflow;
    p.o = *o;
    const dim3 grid((unsigned)(p.tiles_x * p.tiles_y)), block(NTHR);
    hipStream_t s = (hipStream_t)stream;
    if (mode == 1) {
        if (cout > 32) hipLaunchKernelGGL((conv_x3_v5<2, 3, 1>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((conv_x3_v5<1, 3, 1>), grid, block, 0, s, p);
    } else {
        if (cout > 32) hipLaunchKernelGGL((conv_x3_v5<2, 3, 0>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((conv_x3_v5<1, 3, 0>), grid, block, 0, s, p);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
