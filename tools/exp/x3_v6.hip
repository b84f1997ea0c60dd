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

// v6: 256 threads (4 waves, one per SIMD), 16×32 tile, each wave 4 M-tiles × NT N-tiles; ONE LDS stage per workgroup so
// that two workgroups share a CU: while one waits on its chunk's DMA / barrier / epilogue, the other's MFMAs run.
constexpr int NTHR6 = 256, NW6 = 4, MT6 = 4;
template <int NT, int TS, int MODE>
__global__ __launch_bounds__(NTHR6, 2) void conv_x3_v6(X3Params p) {
    constexpr int T = TS * TS;
    constexpr int N = NT * 32;
    constexpr int W_RECS = T * N;
    constexpr int IN_B = IN_RECS * REC;
    constexpr int W_B = W_RECS * REC;
    constexpr int EP_P = 36;                       // restage one 32-channel half at a time
    constexpr int EP_BYTES = TH * TWF * EP_P * 4;  // 73728
    constexpr int LDS_BYTES = IN_B + W_B > EP_BYTES ? IN_B + W_B : EP_BYTES;
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

    auto dma = [&](int j) {
        const int groups = min(16, p.cin - 16 * j) >> 3;
        for (int k = wave; k < IN_RECS / 16; k += NW6) {
            const int r = 16 * k + sub;
            const int s = ps ^ ((r >> 2) & 3);
            const int hy = r / hx, hxi = r - hy * hx;
            const int gy = r0 + hy, gx = x0 + hxi;
            const void *src = g_zero_page;
            if (r < HY * hx && gy < rows_tot && gx < p.W + 2 && (s >> 1) < groups)
                src = p.in + (gy * rowp + gx) * pixb + 64LL * j + (s << 4);
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(lds + k * 1024), 16, 0, 0);
        }
        const unsigned char *wj = p.w + (long long)j * W_B;
        for (int k = wave; k < W_RECS / 16; k += NW6) {
            const int r = 16 * k + sub;
            const int s = ps ^ ((r >> 2) & 3);
            __builtin_amdgcn_global_load_lds((glob_void *)(wj + r * REC + (s << 4)),
                                             (lds_void *)(lds + IN_B + k * 1024), 16, 0, 0);
        }
    };

    int rec0[MT6];
    bool mvalid[MT6];
#pragma unroll
    for (int mt = 0; mt < MT6; ++mt) {
        const int jm = MT6 * wave + mt;
        mvalid[mt] = jm < nmt;
        int q = 32 * jm + ml;
        if (q >= nq) q = 0;
        rec0[mt] = (q / tw) * hx + q % tw;
    }
    const int bsw = (ml >> 2) & 3;
    const int boff = IN_B + ml * REC + (((2 * hl) ^ bsw) << 4);  // hi slot; lo slot = boff ^ 16

    f32x16 acc[MT6][NT];
#pragma unroll
    for (int mt = 0; mt < MT6; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

    for (int j = 0; j < nchunk; ++j) {
        if (j > 0) __syncthreads();  // every wave finished reading the stage
        if (MODE != 1 || j == 0) dma(j);
        __syncthreads();              // chunk j landed
        if (!mvalid[0]) continue;
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int off = (p.tap_y0 + tap / TS) * hx + p.tap_x0 + tap % TS;
            f16x8 ah[MT6], al[MT6], bh[NT], bl[NT];
#pragma unroll
            for (int mt = 0; mt < MT6; ++mt) {
                const int r = rec0[mt] + off;
                const int a = r * REC + (((2 * hl) ^ ((r >> 2) & 3)) << 4);
                ah[mt] = *reinterpret_cast<const f16x8 *>(lds + a);
                al[mt] = *reinterpret_cast<const f16x8 *>(lds + (a ^ 16));
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                bh[nt] = *reinterpret_cast<const f16x8 *>(lds + boff + (tap * N + nt * 32) * REC);
                bl[nt] = *reinterpret_cast<const f16x8 *>(lds + ((boff + (tap * N + nt * 32) * REC) ^ 16));
            }
#pragma unroll
            for (int mt = 0; mt < MT6; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < MT6; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < MT6; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
        }
    }

    // ---- epilogue, one 32-channel half at a time through LDS ----
    const esr_conv_out &o = p.o;
    const long long orow = (long long)(o.out_w + 2);
    float *s_ep = reinterpret_cast<float *>(lds);
    bool ok = true;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        __syncthreads();
#pragma unroll
        for (int mt = 0; mt < MT6; ++mt) {
            if (!mvalid[mt]) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int q = 32 * (MT6 * wave + mt) + (r & 3) + 8 * (r >> 2) + 4 * hl;
                if (q < nq) s_ep[q * EP_P + ml] = acc[mt][nt][r];
            }
        }
        __syncthreads();
        for (int u = tid; u < nq * 4; u += NTHR6) {
            const int q = u >> 2, g = u & 3;
            const int c = 32 * nt + 8 * g;
            if (c >= p.cout) continue;
            const int R = r0 + 1 + q / tw;
            const int b = R / (p.H + 2);
            const int y = R - b * (p.H + 2) - 1;
            if (b >= p.B || y < 0 || y >= p.H) continue;
            const int x = x0 + q % tw;
            const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
            const long long opix = ((long long)b * (o.out_h + 2) + oy + 1) * orow + ox + 1;
            float v[8];
            const f32x4 v0 = *reinterpret_cast<const f32x4 *>(s_ep + q * EP_P + 8 * g);
            const f32x4 v1 = *reinterpret_cast<const f32x4 *>(s_ep + q * EP_P + 8 * g + 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) { v[k] = v0[k]; v[k + 4] = v1[k]; }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const float bk = (c + k < p.cout) ? p.bias[c + k] : 0.f;
                v[k] = v[k] * p.w_scale_inv + bk;
                if (o.lrelu) v[k] = lrelu(v[k]);
            }
            if (o.r1) {
                float rr[8];
                load_group(reinterpret_cast<const unsigned char *>(o.r1) + (opix * o.r1_cp + o.r1_coff + c) * 4, rr);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = o.s1 * v[k] + rr[k];
            }
            if (o.r2) {
                float rr[8];
                load_group(reinterpret_cast<const unsigned char *>(o.r2) + (opix * o.r2_cp + o.r2_coff + c) * 4, rr);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = o.s2 * v[k] + rr[k];
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
    const dim3 grid((unsigned)(p.tiles_x * p.tiles_y)), block(NTHR6);
    hipStream_t s = (hipStream_t)stream;
    if (mode == 1) {
        if (cout > 32) hipLaunchKernelGGL((conv_x3_v6<2, 3, 1>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((conv_x3_v6<1, 3, 1>), grid, block, 0, s, p);
    } else {
        if (cout > 32) hipLaunchKernelGGL((conv_x3_v6<2, 3, 0>), grid, block, 0, s, p);
        else hipLaunchKernelGGL((conv_x3_v6<1, 3, 0>), grid, block, 0, s, p);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
