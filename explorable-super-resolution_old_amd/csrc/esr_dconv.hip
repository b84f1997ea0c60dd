// esr_dconv.hip — convolutions of the patch discriminator on exact-fp32 MFMA, forward and both gradients.
//
// Discriminator_VGG_128_ (architecture.py:222-284) is conv_block(CNA) layers (block.py:129-156) with k = 3 / 4 / 8 / 1,
// stride 1 / 2, zero padding k//2-ish or none, on channels-last tensors.  The D step of optimize_parameters
// (SRRaGAN_model.py:360-433) needs the forward, the data gradient and the weight gradient, and the WGAN-GP penalty
// (loss.py:244-263, autograd.grad(create_graph=True)) differentiates the data gradient again — which is again one of the
// three.  All three are one gather-GEMM over NHWC tensors:
//
//   esr_dconv_fwd    out[b, omy·Y+oay, omx·X+oax, n] = bias[n] + Σ_t Σ_c src[b, smy·Y+offy[t], smx·X+offx[t], c]·w[t][c][n]
//                    M = B·MH·MW output pixels, N = output channels, K = taps × channels; out-of-range source pixels
//                    are the conv's zero padding.  A forward conv is (smy = stride, offy[t] = ky - pad).  The data
//                    gradient of a stride-s conv is s² launches, one per input phase class (cy, cx): a stride-1 gather
//                    over the taps with ky ≡ cy + pad (mod s), written to pixels (s·Y'+cy, s·X'+cx) — the transposed
//                    conv without a zero-stuffed grid.
//   esr_dconv_wgrad  partial[split][t][ci][co] = Σ_{pixels of split} src[.., tap t, ..][ci] · dy[pixel][co]
//                    M = input channels, N = output channels, K = pixels; split-K into `splits` partial slabs that
//                    esr_wgrad_reduce sums in a fixed order (deterministic).
//
// Tiling (fwd): workgroup = 256 threads (4 waves, one per SIMD), 256 pixels × 64 channels; wave w owns M-tiles 2w,
// 2w+1 × two 32-wide N-tiles of v_mfma_f32_32x32x2_f32.  K steps of 32 channels of one tap: the 256 gathered pixel rows
// (128 B each, coalesced per pixel) and the 64×32 weight slab are staged in LDS (row pitch 36 floats: the 16 lanes of a
// ds_read_b128 group hit 16 distinct slots) while the next step is prefetched into registers.  Lane half h consumes
// channels [16h, 16h+16) of the step four at a time (one ds_read_b128 each for A and B, four MFMAs).
// Numerics: v_mfma_f32_32x32x2_f32 is an exact fp32 FMA chain; only the summation order differs from a CPU conv.
#include <hip/hip_runtime.h>
#include "esr_amd.h"
#include "esr_knobs.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glob_void;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__device__ __forceinline__ s16x4 tr_read(const unsigned char *lds, int byte_off) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(lds + byte_off));
}
__device__ __forceinline__ f16x8 cat8(s16x4 a, s16x4 b) {
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}

constexpr int NTH = 256;
constexpr int MT = 256;                  // pixels per workgroup
constexpr int NB = 64;                   // output channels per workgroup
constexpr int KC = 32;                   // channels per K step
constexpr int PS = 36;                   // LDS row pitch (floats)
constexpr int A_IT = MT * KC / 4 / NTH;  // float4 per thread per step: 8
constexpr int B_IT = NB * KC / 4 / NTH;  // 2
constexpr int MAXT = ESR_DCONV_MAX_TAPS;

struct FwdParams {
    const float *src;
    int B, Hs, Ws, sp, kc, vec;  // source NHWC [B][Hs][Ws][sp], channels [0, kc); vec: 16-B loads allowed
    const float *w;              // packed [T][nck][n_pad][32]
    int nck, n_pad;
    const float *bias;           // [n] or null
    float *out;
    int Ho, Wo, op, n;           // out NHWC [B][Ho][Wo][op], channels [0, n)
    int MH, MW;
    int omy, oay, omx, oax, smy, smx;
    int T;
    int offy[MAXT], offx[MAXT];
    float *partial;  // split-K (x3 kernel, gridDim.z > 1): [z][M][n_pad] raw sums, reduced by dconv_splitk_reduce
    const unsigned char *wsx;  // pre-split x3 weights (include/esr_amd.h esr_dconv_fwd_sd w_split) or null
    const int32_t *wexp;       // their power-of-two exponent E (the stored values are w·2^E)
    int s2c, s2pad, s2g, s2sh;  // > 0: space-to-depth source (src_quad), channel group s2g = 2^s2sh (s2sh < 0: not
    int d2c, d2pad, d2g, d2sh;  // a power of two); d2*: depth-to-space output (put_out); 0: plain
};

__device__ __forceinline__ f32x4 load4(const float *row, int c, int kc, bool vec) {
    if (vec && c + 4 <= kc) return *reinterpret_cast<const f32x4 *>(row + c);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (c + e < kc) v[e] = row[c + e];
    return v;
}

// The 4-channel quad from channel c of gather point (sy, sx) of image b; zero outside the image (the conv's padding).
// s2c > 0: the source is the space-to-depth view of a stride-2 conv's input (esr_dconv_fwd_sd): virtual channel
// c = (c' / G)·4G + (2·py + px)·G + c' % G of virtual pixel (sy, sx) is channel c' of real pixel
// (2·sy + py - s2pad, 2·sx + px - s2pad) of the [B][Hs][Ws][sp] source, G = s2g (32 where s2c % 32 == 0, so that a
// 32-channel K chunk is 128 contiguous bytes of one real pixel; else s2c).  s2c % 4 == 0: a quad never straddles
// two phases.
__device__ __forceinline__ f32x4 src_quad(const FwdParams &p, int b, int sy, int sx, int c, bool vec) {
    int kc = p.kc;
    if (p.s2c) {
        int ph;
        if (p.s2sh >= 0) {  // shifts: this runs for every staged quad
            ph = (c >> p.s2sh) & 3;
            c = ((c >> (p.s2sh + 2)) << p.s2sh) | (c & (p.s2g - 1));
        } else {
            ph = (c / p.s2g) & 3;
            c = (c / (4 * p.s2g)) * p.s2g + c % p.s2g;
        }  // (past the last group — kc padding — c >= s2c: reads as zero below)
        sy = 2 * sy + (ph >> 1) - p.s2pad;
        sx = 2 * sx + (ph & 1) - p.s2pad;
        kc = p.s2c;
    }
    if (c < kc && sy >= 0 && sy < p.Hs && sx >= 0 && sx < p.Ws)
        return load4(p.src + (((long long)b * p.Hs + sy) * p.Ws + sx) * p.sp, c, kc, vec);
    return f32x4{0.f, 0.f, 0.f, 0.f};
}

// out at output grid point (Y, X), channel n.  d2c > 0: depth-to-space (the data gradient of a stride-2 conv in its
// space-to-depth form): channel n = (c' / G)·4G + (2·py + px)·G + c' % G of grid point (Y, X) (G = d2g, the
// grouping of src_quad) is channel c' of real pixel (2·(omy·Y + oay) + py - d2pad, 2·(omx·X + oax) + px - d2pad);
// pixels outside [0, Ho) × [0, Wo) (the padding border) are dropped.
__device__ __forceinline__ void put_out(const FwdParams &p, int b, int Y, int X, int n, float v) {
    int oy = p.omy * Y + p.oay, ox = p.omx * X + p.oax;
    if (p.d2c) {
        int ph;
        if (p.d2sh >= 0) {  // shifts: this runs for every output element
            ph = (n >> p.d2sh) & 3;
            n = ((n >> (p.d2sh + 2)) << p.d2sh) | (n & (p.d2g - 1));
        } else {
            ph = (n / p.d2g) & 3;
            n = (n / (4 * p.d2g)) * p.d2g + n % p.d2g;
        }
        oy = 2 * oy + (ph >> 1) - p.d2pad;
        ox = 2 * ox + (ph & 1) - p.d2pad;
        if (oy < 0 || oy >= p.Ho || ox < 0 || ox >= p.Wo) return;
    }
    p.out[(((long long)b * p.Ho + oy) * p.Wo + ox) * p.op + n] = v;
}

__global__ __launch_bounds__(NTH, 2) void dconv_fwd_kernel(FwdParams p) {
    __shared__ __attribute__((aligned(16))) float lds[(MT + NB) * PS];
    float *s_a = lds, *s_b = lds + MT * PS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ml = lane & 31;
    const int per_img = p.MH * p.MW;
    const long long M = (long long)p.B * per_img;
    const long long m0 = (long long)blockIdx.x * MT;
    const int n0 = blockIdx.y * NB;
    const int cg = tid & 7;  // this thread's 4-channel group of every staged pixel row
    const bool vec = p.vec != 0;

    int pb[A_IT], py[A_IT], px[A_IT];
#pragma unroll
    for (int k = 0; k < A_IT; ++k) {
        const long long m = m0 + (tid >> 3) + 32 * k;
        pb[k] = -1;
        py[k] = 0;
        px[k] = 0;
        if (m < M) {
            const int b = (int)(m / per_img), r = (int)(m - (long long)b * per_img);
            pb[k] = b;
            py[k] = r / p.MW;
            px[k] = r - py[k] * p.MW;
        }
    }
    f32x4 ra[A_IT], rb[B_IT];
    const int nsteps = p.T * p.nck;
    auto load = [&](int step) {
        const int t = step / p.nck, j = step - t * p.nck;
        const int c = j * KC + cg * 4;
        const int oy = p.offy[t], ox = p.offx[t];
#pragma unroll
        for (int k = 0; k < A_IT; ++k) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (pb[k] >= 0) v = src_quad(p, pb[k], p.smy * py[k] + oy, p.smx * px[k] + ox, c, vec);
            ra[k] = v;
        }
        const float *wj = p.w + ((long long)(t * p.nck + j) * p.n_pad + n0) * KC;
#pragma unroll
        for (int k = 0; k < B_IT; ++k) rb[k] = *reinterpret_cast<const f32x4 *>(wj + (tid + k * NTH) * 4);
    };
    auto store = [&]() {
#pragma unroll
        for (int k = 0; k < A_IT; ++k) *reinterpret_cast<f32x4 *>(s_a + ((tid >> 3) + 32 * k) * PS + cg * 4) = ra[k];
#pragma unroll
        for (int k = 0; k < B_IT; ++k) {
            const int idx = tid + k * NTH;
            *reinterpret_cast<f32x4 *>(s_b + (idx >> 3) * PS + (idx & 7) * 4) = rb[k];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

    load(0);
    for (int step = 0; step < nsteps; ++step) {
        __syncthreads();
        store();
        __syncthreads();
        if (step + 1 < nsteps) load(step + 1);
        const float *a0 = s_a + (64 * wave + ml) * PS + 16 * hl;
        const float *a1 = a0 + 32 * PS;
        const float *b0 = s_b + ml * PS + 16 * hl;
        const float *b1 = b0 + 32 * PS;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const f32x4 av0 = *reinterpret_cast<const f32x4 *>(a0 + 4 * g);
            const f32x4 av1 = *reinterpret_cast<const f32x4 *>(a1 + 4 * g);
            const f32x4 bv0 = *reinterpret_cast<const f32x4 *>(b0 + 4 * g);
            const f32x4 bv1 = *reinterpret_cast<const f32x4 *>(b1 + 4 * g);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av0[s], bv0[s], acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av0[s], bv1[s], acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av1[s], bv0[s], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av1[s], bv1[s], acc[1][1], 0, 0, 0);
            }
        }
    }

    // D layout (32x32 f32 MFMA): lane holds column n = lane & 31, rows m = (r&3) + 8(r>>2) + 4(lane>>5); the output
    // pixel of each row is decoded once for all N-tiles (32-bit: M < 2^31 is checked at launch)
    float bn[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
        const int n = n0 + nt * 32 + ml;
        bn[nt] = (p.bias && n < p.n) ? p.bias[n] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = (int)m0 + 64 * wave + 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * hl;
            if (m >= (int)M) continue;
            const int b = m / per_img, rr = m - b * per_img;
            const int Y = rr / p.MW, X = rr - Y * p.MW;
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) {
                const int n = n0 + nt * 32 + ml;
                if (n < p.n) put_out(p, b, Y, X, n, acc[mt][nt][r] + bn[nt]);
            }
        }
}

// ---- halo-tile forward (exact fp32, the default) -----------------------------------------------------------------------
// The same gather-GEMM, but a workgroup owns a 2-D output tile (TY rows × 32 columns of the MH × MW grid of one image)
// instead of 256 pixel-linear outputs, so the source pixels of ALL taps of a 32-channel chunk are one halo window that
// is staged in LDS once per chunk: IY = smy·(TY-1) + span_y + 1 rows × (smx·31 + span_x + 1) columns (span = max - min
// tap offset).  The gather kernel re-stages the 256 source rows of every (tap, chunk) step: 9 / 16 / 64 × the rows for
// the 3×3 / 4×4 / 8×8 convolutions, which made it L2→LDS-staging-bound at ≈half the f32 MFMA rate.
// Stride-2 sources (the 4×4 s2 forward) are stored de-interleaved by column parity (parity-major, then half-column), so
// the 32 lanes of a fragment read consecutive LDS pixels for every tap: pixel pitch 36 floats → the 16 lanes of a
// ds_read_b128 group hit 16 distinct 4-bank slots.  The weights of one (tap, chunk) step (64 output channels × 32)
// are prefetched into registers during the previous step and staged through a small LDS slab, as the gather kernel.
// Wave w of 4 owns WM M-tiles (output rows) × WN N-tiles (32 channels) of v_mfma_f32_32x32x2_f32; TY = 2·WM·WN.
// Split-K (gridDim.z > 1) divides the chunks; the raw sums go to `partial` for dconv_splitk_reduce.
struct HaloParams {
    int TY, tiles_x, tiles_y;  // tile rows; tiles per image row / column
    int IY, IXp, npar, IXt;    // halo rows; columns per parity; parities (= smx); IXt = npar·IXp
    int oymin, oxmin;          // smallest tap offsets
    int b_off;                 // byte offset of the weight slab in LDS
    int cw;                    // tile columns (32; 16: two rows per M-tile, dconv_fwd_halo_x_kernel CW)
};

template <int WM, int WN>
__global__ __launch_bounds__(NTH, 2) void dconv_fwd_halo_kernel(FwdParams p, HaloParams h) {
    constexpr int TY = 2 * WM * WN, MW_ = TY / WM;  // waves along M
    extern __shared__ __attribute__((aligned(16))) float dlds[];
    float *s_a = dlds, *s_b = dlds + h.b_off / 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ml = lane & 31;
    int id = blockIdx.x;
    const int txi = id % h.tiles_x;
    id /= h.tiles_x;
    const int tyi = id % h.tiles_y, b = id / h.tiles_y;
    const int Y0 = tyi * TY, X0 = txi * 32;
    const int n0 = blockIdx.y * NB;
    const int wm = wave % MW_, wn = wave / MW_;
    const bool vec = p.vec != 0;
    const int sy0 = p.smy * Y0 + h.oymin, sx0 = p.smx * X0 + h.oxmin;
    const int c_begin = (int)((long long)p.nck * blockIdx.z / gridDim.z);
    const int c_end = (int)((long long)p.nck * (blockIdx.z + 1) / gridDim.z);
    const int nsteps = (c_end - c_begin) * p.T;

    f32x4 rb[B_IT];
    auto load_b = [&](int step) {
        const int j = c_begin + step / p.T, t = step - (step / p.T) * p.T;
        const float *wj = p.w + ((long long)(t * p.nck + j) * p.n_pad + n0) * KC;
#pragma unroll
        for (int k = 0; k < B_IT; ++k) rb[k] = *reinterpret_cast<const f32x4 *>(wj + (tid + k * NTH) * 4);
    };
    // the halo window of chunk j: every thread stages (pixel, 4-channel quad) items, 8 loads in flight at a time
    auto stage_a = [&](int j) {
        const int total = h.IY * h.IXt * 8;
        for (int base = 0; base < total; base += 8 * NTH) {
            f32x4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int idx = base + u * NTH + tid;
                v[u] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (idx < total) {
                    const int pix = idx >> 3, q = idx & 7;
                    const int r = pix / h.IXt, cc = pix - r * h.IXt;
                    const int par = cc / h.IXp, hc = cc - par * h.IXp;
                    v[u] = src_quad(p, b, sy0 + r, sx0 + hc * h.npar + par, j * KC + 4 * q, vec);
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int idx = base + u * NTH + tid;
                if (idx < total) *reinterpret_cast<f32x4 *>(s_a + (idx >> 3) * PS + 4 * (idx & 7)) = v[u];
            }
        }
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int k = 0; k < WN; ++k)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;

    if (nsteps > 0) load_b(0);
    for (int step = 0; step < nsteps; ++step) {
        const int t = step % p.T;
        __syncthreads();
        if (t == 0) stage_a(c_begin + step / p.T);
#pragma unroll
        for (int k = 0; k < B_IT; ++k) {
            const int idx = tid + k * NTH;
            *reinterpret_cast<f32x4 *>(s_b + (idx >> 3) * PS + (idx & 7) * 4) = rb[k];
        }
        __syncthreads();
        if (step + 1 < nsteps) load_b(step + 1);
        const int dy = p.offy[t] - h.oymin, dx = p.offx[t] - h.oxmin;
        const int col = (h.npar == 1) ? ml + dx : (dx & 1) * h.IXp + ml + (dx >> 1);
        const float *a_base[WM];
#pragma unroll
        for (int i = 0; i < WM; ++i) {
            const int ty = wm * WM + i;
            a_base[i] = s_a + ((p.smy * ty + dy) * h.IXt + col) * PS + 16 * hl;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            f32x4 av[WM], bv[WN];
#pragma unroll
            for (int i = 0; i < WM; ++i) av[i] = *reinterpret_cast<const f32x4 *>(a_base[i] + 4 * g);
#pragma unroll
            for (int k = 0; k < WN; ++k)
                bv[k] = *reinterpret_cast<const f32x4 *>(s_b + ((wn * WN + k) * 32 + ml) * PS + 16 * hl + 4 * g);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < WM; ++i)
#pragma unroll
                    for (int k = 0; k < WN; ++k)
                        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][s], bv[k][s], acc[i][k], 0, 0, 0);
        }
    }

    // D layout (32x32 f32 MFMA): lane holds column n = lane & 31, rows m = (r&3) + 8(r>>2) + 4(lane>>5) = X - X0
    const long long per_img = (long long)p.MH * p.MW;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
        const int Y = Y0 + wm * WM + i;
        if (Y >= p.MH) continue;
#pragma unroll
        for (int k = 0; k < WN; ++k) {
            const int nl = (wn * WN + k) * 32 + ml, n = n0 + nl;
            if (gridDim.z > 1) {  // raw partial sums, pixel-linear; bias and the output map are the reduction's
                float *part = p.partial + (long long)blockIdx.z * p.B * per_img * p.n_pad;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int X = X0 + (r & 3) + 8 * (r >> 2) + 4 * hl;
                    if (X < p.MW) part[(b * per_img + (long long)Y * p.MW + X) * p.n_pad + n] = acc[i][k][r];
                }
                continue;
            }
            if (n >= p.n) continue;
            const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int X = X0 + (r & 3) + 8 * (r >> 2) + 4 * hl;
                if (X < p.MW) put_out(p, b, Y, X, n, acc[i][k][r] + bn);
            }
        }
    }
}

// ---- x3 forward (split-f16 operands, fp32-level accuracy) -------------------------------------------------------------
// The same gather-GEMM on v_mfma_f32_32x32x16_f16: every staged fp32 operand value v is carried as hi = f16(v·s),
// lo = f16(v·s - hi) and a product as a_hi·b_hi + a_hi·b_lo + a_lo·b_hi (esr_conv_x3.hip's scheme), with the split
// done here at staging (the operands are PyTorch-produced fp32 tensors: activations, gradients, or gradients of
// gradients in the WGAN-GP double backward).  Scales: per K step (one tap × 32 channels) the workgroup takes the max
// |a| of its 256 × 32 A tile and max |b| of its 64 × 32 B tile; s_a = 2^eA, s_b = 2^eB bring each max into
// [2^13, 2^14), so tiny gradients (~1e-9) sit in f16's normal range like activations do.  The accumulators hold the
// sum in the scale 2^(eA + eB) of the current step and are multiplied by 2^(new - old) when it changes (v_ldexp:
// exact), by 2^-(eA + eB) at the end.  LDS rows: 32 f16 hi then 32 f16 lo (128 B) + 16 B pad: the 16 rows of a
// ds_read_b128 group land on 16 distinct 4-bank slots.
// x6 (NP = 3 pieces): a third f16 piece lo2 = f16(v·s - hi - lo) and the products hi·hi + hi·lo + lo·hi + lo·lo +
// hi·lo2 + lo2·hi — each operand carried to ~33 bits, every dropped term below 2^-33 of the step's scale, so the
// result is an fp32 FMA chain's up to the fp32 accumulation itself (x3 drops lo·lo and carries 22 bits: ~2^-22 per
// product).  Rows: 32 hi, 32 lo, 32 lo2 (f16) + 16 B pad = 208 B = 52 dwords, so the 16 rows of a ds_read_b128
// group still land on 16 distinct 4-bank slots.
template <int NP> struct XPitch { static constexpr int v = NP == 2 ? 144 : 208; };

__device__ __forceinline__ int tile_exp(float m, int e_keep) {
    if (!(m > 0.f) || !(m <= 3.4e38f)) return e_keep;  // all zero, or NaN / inf (propagates unscaled)
    int ex;
    frexpf(m, &ex);
    return 14 - ex;
}

// NBX = 64 or 128 output channels per workgroup (128: the A tile, re-gathered per tap, feeds twice the MFMAs)
template <int NBX, int NP>
__global__ __launch_bounds__(NTH, 2) void dconv_fwd_x3_kernel(FwdParams p) {
    constexpr int NTN = NBX / 32, BX_IT = NBX * KC / 4 / NTH, XP = XPitch<NP>::v;
    __shared__ __attribute__((aligned(16))) unsigned char lds[(MT + NBX) * XP];
    __shared__ float s_red[2][2][NTH / 64];
    unsigned char *s_a = lds, *s_b = lds + MT * XP;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ml = lane & 31;
    const int per_img = p.MH * p.MW;
    const long long M = (long long)p.B * per_img;
    const long long m0 = (long long)blockIdx.x * MT;
    const int n0 = blockIdx.y * NBX;
    const int cg = tid & 7;
    const bool vec = p.vec != 0;

    int pb[A_IT], py[A_IT], px[A_IT];
#pragma unroll
    for (int k = 0; k < A_IT; ++k) {
        const long long m = m0 + (tid >> 3) + 32 * k;
        pb[k] = -1;
        py[k] = 0;
        px[k] = 0;
        if (m < M) {
            const int b = (int)(m / per_img), r = (int)(m - (long long)b * per_img);
            pb[k] = b;
            py[k] = r / p.MW;
            px[k] = r - py[k] * p.MW;
        }
    }
    f32x4 ra[A_IT], rb[BX_IT];
    // split-K: workgroup z of gridDim.z takes K steps [s_begin, s_end)
    const int nsteps_all = p.T * p.nck;
    const int s_begin = (int)((long long)nsteps_all * blockIdx.z / gridDim.z);
    const int s_end = (int)((long long)nsteps_all * (blockIdx.z + 1) / gridDim.z);
    auto load = [&](int step) {
        const int t = step / p.nck, j = step - t * p.nck;
        const int c = j * KC + cg * 4;
        const int oy = p.offy[t], ox = p.offx[t];
#pragma unroll
        for (int k = 0; k < A_IT; ++k) {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (pb[k] >= 0) v = src_quad(p, pb[k], p.smy * py[k] + oy, p.smx * px[k] + ox, c, vec);
            ra[k] = v;
        }
        const float *wj = p.w + ((long long)(t * p.nck + j) * p.n_pad + n0) * KC;
#pragma unroll
        for (int k = 0; k < BX_IT; ++k) rb[k] = *reinterpret_cast<const f32x4 *>(wj + (tid + k * NTH) * 4);
    };
    auto publish = [&](int slot) {
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int k = 0; k < A_IT; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) ma = fmaxf(ma, fabsf(ra[k][e]));
#pragma unroll
        for (int k = 0; k < BX_IT; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) mb = fmaxf(mb, fabsf(rb[k][e]));
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) {
            ma = fmaxf(ma, __shfl_xor(ma, s));
            mb = fmaxf(mb, __shfl_xor(mb, s));
        }
        if (lane == 0) {
            s_red[slot][0][wave] = ma;
            s_red[slot][1][wave] = mb;
        }
    };
    auto put = [&](unsigned char *row, f32x4 v, float s) {  // 4 channels at quad cg of a staged row
        f16x4 h, l, l2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float x = v[e] * s;
            h[e] = (_Float16)x;
            const float r = x - (float)h[e];
            l[e] = (_Float16)r;
            if (NP == 3) l2[e] = (_Float16)(r - (float)l[e]);
        }
        *reinterpret_cast<f16x4 *>(row + cg * 8) = h;
        *reinterpret_cast<f16x4 *>(row + 64 + cg * 8) = l;
        if (NP == 3) *reinterpret_cast<f16x4 *>(row + 128 + cg * 8) = l2;
    };

    f32x16 acc[2][NTN];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;
    int ea = 0, eb = 0;

    if (s_begin < s_end) {
        load(s_begin);
        publish(0);
    }
    for (int step = s_begin; step < s_end; ++step) {
        __syncthreads();
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int w = 0; w < NTH / 64; ++w) {
            ma = fmaxf(ma, s_red[(step - s_begin) & 1][0][w]);
            mb = fmaxf(mb, s_red[(step - s_begin) & 1][1][w]);
        }
        const int ea2 = tile_exp(ma, ea), eb2 = tile_exp(mb, eb);
        if (ea2 + eb2 != ea + eb) {
            const int d = ea2 + eb2 - ea - eb;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[mt][nt][r] = ldexpf(acc[mt][nt][r], d);
        }
        ea = ea2;
        eb = eb2;
        const float sa = ldexpf(1.f, ea), sb = ldexpf(1.f, eb);
#pragma unroll
        for (int k = 0; k < A_IT; ++k) put(s_a + ((tid >> 3) + 32 * k) * XP, ra[k], sa);
#pragma unroll
        for (int k = 0; k < BX_IT; ++k) put(s_b + ((tid + k * NTH) >> 3) * XP, rb[k], sb);
        __syncthreads();
        if (step + 1 < s_end) load(step + 1);
        const unsigned char *a0 = s_a + (64 * wave + ml) * XP + 16 * hl;
        const unsigned char *b0 = s_b + ml * XP + 16 * hl;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            f16x8 ah[2], al[2], al2[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                ah[i] = *reinterpret_cast<const f16x8 *>(a0 + i * 32 * XP + 32 * s);
                al[i] = *reinterpret_cast<const f16x8 *>(a0 + i * 32 * XP + 64 + 32 * s);
                if (NP == 3) al2[i] = *reinterpret_cast<const f16x8 *>(a0 + i * 32 * XP + 128 + 32 * s);
            }
#pragma unroll
            for (int nt = 0; nt < NTN; ++nt) {
                const f16x8 bh = *reinterpret_cast<const f16x8 *>(b0 + nt * 32 * XP + 32 * s);
                const f16x8 bl = *reinterpret_cast<const f16x8 *>(b0 + nt * 32 * XP + 64 + 32 * s);
                f16x8 bl2;
                if (NP == 3) bl2 = *reinterpret_cast<const f16x8 *>(b0 + nt * 32 * XP + 128 + 32 * s);
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    if (NP == 3) {  // smallest terms first
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al2[mt], bh, acc[mt][nt], 0, 0, 0);
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bl2, acc[mt][nt], 0, 0, 0);
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mt], bl, acc[mt][nt], 0, 0, 0);
                    }
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mt], bh, acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bl, acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bh, acc[mt][nt], 0, 0, 0);
                }
            }
        }
        if (step + 1 < s_end) publish((step + 1 - s_begin) & 1);
    }

    if (gridDim.z > 1) {  // raw partial sums, pixel-linear; bias and the output map are the reduction's
        float *part = p.partial + (long long)blockIdx.z * M * p.n_pad;
#pragma unroll
        for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const long long m = m0 + 64 * wave + 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * hl;
                    if (m < M) part[m * p.n_pad + n0 + nt * 32 + ml] = ldexpf(acc[mt][nt][r], -(ea + eb));
                }
        return;
    }
    float bn[NTN];  // the output pixel of each row is decoded once for all N-tiles (32-bit: M < 2^31 at launch)
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt) {
        const int n = n0 + nt * 32 + ml;
        bn[nt] = (p.bias && n < p.n) ? p.bias[n] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = (int)m0 + 64 * wave + 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * hl;
            if (m >= (int)M) continue;
            const int b = m / per_img, rr = m - b * per_img;
            const int Y = rr / p.MW, X = rr - Y * p.MW;
#pragma unroll
            for (int nt = 0; nt < NTN; ++nt) {
                const int n = n0 + nt * 32 + ml;
                if (n < p.n) put_out(p, b, Y, X, n, ldexpf(acc[mt][nt][r], -(ea + eb)) + bn[nt]);
            }
        }
}


// ---- halo-tile forward, split precision (x3 / x6) ---------------------------------------------------------------------
// dconv_fwd_halo_kernel's tiling (the source window of all taps of a 32-channel chunk staged once) with the operands in
// NP f16 pieces (x3: hi, lo; x6: hi, lo, lo2) as dconv_fwd_x3_kernel.  Scales: per chunk the workgroup's max |a| over
// the halo window (a first pass over the window's global loads, values discarded; the second pass scales, splits and
// stores), per (tap, chunk) step the max |b| of the weight slab; the accumulators are rescaled exactly whenever the
// sum of the two exponents changes.
// NBX = 64 or 128 output channels per workgroup (128: each wave 4 N-tiles, twice the MFMAs per staged B slab and A
// fragment; taken for x3 where n_pad allows and the grid still fills the chip).  TY = WM·WN·128 / NBX rows.
// DBG (experiment build only, garbage outputs): 1 = no weight-slab staging (no loads, max, split, stores; one barrier
// per chunk), 2 = no fragment reads / MFMAs, 4 = the halo window staged for the first chunk only
// CW = 16: an M-tile is 2 rows × 16 columns (stride-1 sources only), for grids whose width 32-column tiles would cover
// with > 30 % waste (the 38-wide conv2_1 / fc8 layers at config 3); a tile is then 2·TY rows × 16 columns.
// PB (x3 only): the weights come pre-split (esr_dconv_fwd_sd w_split: hi/lo f16 at one power-of-two scale 2^E per
// tensor, each 128-byte (t, chunk, n) row's 16-B slots XOR-swizzled by (n >> 1) & 7 so that a linear copy gives a
// conflict-free LDS image) and are LDS-DMA'd into two slots, the next step's under the current step's MFMAs: no weight
// loads through registers, no per-step max / split / rescale, one barrier per step instead of two.
template <int WM, int WN, int NP, int NBX = NB, int DBG = 0, int OCC = 2, int CW = 32, bool PB = false>
__global__ __launch_bounds__(NTH, OCC) void dconv_fwd_halo_x_kernel(FwdParams p, HaloParams h) {
    constexpr int TY = WM * WN * 128 / NBX, MWV = TY / WM, XPn = XPitch<NP>::v, BX_IT = NBX * KC / 4 / NTH;
    static_assert(!PB || (NP == 2 && DBG == 0), "pre-split weights: x3");
    constexpr int RBB = 128, SLOT = NBX * RBB;  // PB: bytes per weight row / per step's slab
    constexpr int RPM = 32 / CW;  // output rows per M-tile
    static_assert((TY / WM) * (NBX / 32 / WN) == NTH / 64, "waves along M x waves along N = 4");
    extern __shared__ __attribute__((aligned(16))) unsigned char xlds[];
    __shared__ float s_reda[NTH / 64], s_redb[2][NTH / 64];  // per-wave max of the halo / of the weight slab
    unsigned char *s_a = xlds, *s_b = xlds + h.b_off;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ml = lane & 31;
    int id = blockIdx.x;
    const int txi = id % h.tiles_x;
    id /= h.tiles_x;
    const int tyi = id % h.tiles_y, b = id / h.tiles_y;
    const int Y0 = tyi * TY * RPM, X0 = txi * CW;
    const int n0 = blockIdx.y * NBX;
    const int wm = wave % MWV, wn = wave / MWV;
    const bool vec = p.vec != 0;
    const int sy0 = p.smy * Y0 + h.oymin, sx0 = p.smx * X0 + h.oxmin;
    const int c_begin = (int)((long long)p.nck * blockIdx.z / gridDim.z);
    const int c_end = (int)((long long)p.nck * (blockIdx.z + 1) / gridDim.z);
    const int nsteps = (c_end - c_begin) * p.T;

    auto split_put = [&](unsigned char *row, int q, f32x4 v, float sc) {  // 4 channels at quad q of a staged row
        f16x4 hi, lo, lo2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float x = v[e] * sc;
            hi[e] = (_Float16)x;
            const float r = x - (float)hi[e];
            lo[e] = (_Float16)r;
            if (NP == 3) lo2[e] = (_Float16)(r - (float)lo[e]);
        }
        *reinterpret_cast<f16x4 *>(row + q * 8) = hi;
        *reinterpret_cast<f16x4 *>(row + 64 + q * 8) = lo;
        if (NP == 3) *reinterpret_cast<f16x4 *>(row + 128 + q * 8) = lo2;
    };
    auto halo_item = [&](int idx, int j) -> f32x4 {
        const int pix = idx >> 3, q = idx & 7;
        const int r = pix / h.IXt, cc = pix - r * h.IXt;
        const int par = cc / h.IXp, hc = cc - par * h.IXp;
        return src_quad(p, b, sy0 + r, sx0 + hc * h.npar + par, j * KC + 4 * q, vec);
    };
    auto wave_max = [&](float m) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        return m;
    };
    // stage chunk j's halo window: one pass over global memory — each item's fp32 quad goes into its row of the LDS
    // image (a staged row's 128 fp32 bytes fit in its split pitch) while the max |a| is taken; after the cross-wave
    // max each thread converts whole rows in place (all 8 quads read before any write), so the window is not read
    // from L2 twice (the two-pass form cost up to 40 % of a space-to-depth launch: profiles/r3_halo_split.txt)
    const int total_a = h.IY * h.IXt * 8;  // fp32 quads of a chunk's halo window
    // PB: the next chunk's window is loaded into registers during the last step of the current one when it fits
    // quads per thread (48 VGPRs); not where the registers run out (128-wide N tiles, three workgroups per CU: spills)
    constexpr int PFQ = (PB && OCC == 2 && NBX == 64) ? 12 : 0;
    const bool pf_ok = PFQ > 0 && total_a <= PFQ * NTH;
    f32x4 pf[PFQ > 0 ? PFQ : 1];
    auto prefetch_a = [&](int j) {
#pragma unroll
        for (int u = 0; u < PFQ; ++u) {
            const int idx = u * NTH + tid;
            pf[u] = idx < total_a ? halo_item(idx, j) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    // stage chunk j's window (or, from_pf, the prefetched one) and split it; returns its exponent
    auto stage_a = [&](int j, int e_keep, bool from_pf = false) {
        const int total = total_a;
        float m = 0.f;
        if (from_pf) {
#pragma unroll
            for (int u = 0; u < PFQ; ++u) {
                const int idx = u * NTH + tid;
#pragma unroll
                for (int e = 0; e < 4; ++e) m = fmaxf(m, fabsf(pf[u][e]));
                if (idx < total) *reinterpret_cast<f32x4 *>(s_a + (idx >> 3) * XPn + (idx & 7) * 16) = pf[u];
            }
        } else {
            for (int base = 0; base < total; base += 8 * NTH) {
                f32x4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int idx = base + u * NTH + tid;
                    v[u] = idx < total ? halo_item(idx, j) : f32x4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int idx = base + u * NTH + tid;
#pragma unroll
                    for (int e = 0; e < 4; ++e) m = fmaxf(m, fabsf(v[u][e]));
                    if (idx < total) *reinterpret_cast<f32x4 *>(s_a + (idx >> 3) * XPn + (idx & 7) * 16) = v[u];
                }
            }
        }
        m = wave_max(m);
        if (lane == 0) s_reda[wave] = m;
        __syncthreads();
        float mm = 0.f;
#pragma unroll
        for (int w = 0; w < NTH / 64; ++w) mm = fmaxf(mm, s_reda[w]);
        const int ea = tile_exp(mm, e_keep);
        const float sc = ldexpf(1.f, ea);
        const int rows = h.IY * h.IXt;
        for (int r = tid; r < rows; r += NTH) {
            unsigned char *row = s_a + r * XPn;
            f32x4 q[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) q[k] = *reinterpret_cast<const f32x4 *>(row + 16 * k);
#pragma unroll
            for (int k = 0; k < 8; ++k) split_put(row, k, q[k], sc);
        }
        return ea;
    };

    f32x4 rb[BX_IT];
    auto load_b = [&](int step) {
        const int j = c_begin + step / p.T, t = step - (step / p.T) * p.T;
        const float *wj = p.w + ((long long)(t * p.nck + j) * p.n_pad + n0) * KC;
#pragma unroll
        for (int k = 0; k < BX_IT; ++k) rb[k] = *reinterpret_cast<const f32x4 *>(wj + (tid + k * NTH) * 4);
    };
    auto publish_b = [&](int slot) {
        float mb = 0.f;
#pragma unroll
        for (int k = 0; k < BX_IT; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) mb = fmaxf(mb, fabsf(rb[k][e]));
        mb = wave_max(mb);
        if (lane == 0) s_redb[slot][wave] = mb;
    };

    f32x16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int k = 0; k < WN; ++k)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][k][r] = 0.f;
    int ea = 0, eb = 0;

    if constexpr (PB) {
        eb = *p.wexp;
        auto dma_b = [&](int step, int slot) {  // the step's NBX weight rows: one linear copy
            const int j = c_begin + step / p.T, t = step - (step / p.T) * p.T;
            const unsigned char *src = p.wsx + ((long long)(t * p.nck + j) * p.n_pad + n0) * RBB + 16 * lane;
#pragma unroll
            for (int q = wave; q < SLOT / 1024; q += NTH / 64)
                __builtin_amdgcn_global_load_lds((glob_void *)(src + q * 1024),
                                                 (lds_void *)(s_b + slot * SLOT + q * 1024), 16, 0, 0);
        };
        if (nsteps > 0) dma_b(0, 0);
        for (int step = 0; step < nsteps; ++step) {
            const int t = step % p.T;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's copy of the step's weights landed
            __syncthreads();  // every copy landed; every wave is done with step - 1 (its slot, and the window at t 0)
            if (t == 0) {
                const int ea2 = stage_a(c_begin + step / p.T, ea, pf_ok && step > 0);  // (contains a barrier)
                __syncthreads();                                                       // the split window is in place
                if (ea2 != ea) {
#pragma unroll
                    for (int i = 0; i < WM; ++i)
#pragma unroll
                        for (int k = 0; k < WN; ++k)
#pragma unroll
                            for (int r = 0; r < 16; ++r) acc[i][k][r] = ldexpf(acc[i][k][r], ea2 - ea);
                    ea = ea2;
                }
            }
            if (step + 1 < nsteps) dma_b(step + 1, (step + 1) & 1);  // lands under this step's MFMAs
            if (pf_ok && t == p.T - 1 && step + 1 < nsteps) prefetch_a(c_begin + (step + 1) / p.T);  // next window
            const int dy = p.offy[t] - h.oymin, dx = p.offx[t] - h.oxmin;
            const int mc = ml % CW, mr = ml / CW;
            const int col = (h.npar == 1) ? mc + dx : (dx & 1) * h.IXp + mc + (dx >> 1);
            const unsigned char *a_base[WM];
#pragma unroll
            for (int i = 0; i < WM; ++i) {
                const int ty = wm * WM + i;
                a_base[i] = s_a + ((p.smy * (RPM * ty + mr) + dy) * h.IXt + col) * XPn + 16 * hl;
            }
            const unsigned char *bslot = s_b + (step & 1) * SLOT;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                f16x8 ah[WM], al[WM];
#pragma unroll
                for (int i = 0; i < WM; ++i) {
                    ah[i] = *reinterpret_cast<const f16x8 *>(a_base[i] + 32 * s2);
                    al[i] = *reinterpret_cast<const f16x8 *>(a_base[i] + 64 + 32 * s2);
                }
#pragma unroll
                for (int k = 0; k < WN; ++k) {
                    const int n = (wn * WN + k) * 32 + ml, sw = (n >> 1) & 7;
                    const unsigned char *brow = bslot + n * RBB;
                    const f16x8 bh = *reinterpret_cast<const f16x8 *>(brow + (((2 * s2 + hl) ^ sw) << 4));
                    const f16x8 bl = *reinterpret_cast<const f16x8 *>(brow + (((4 + 2 * s2 + hl) ^ sw) << 4));
#pragma unroll
                    for (int i = 0; i < WM; ++i) {
                        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, acc[i][k], 0, 0, 0);
                        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl, acc[i][k], 0, 0, 0);
                        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh, acc[i][k], 0, 0, 0);
                    }
                }
            }
        }
    }

    if (!PB && nsteps > 0 && !(DBG & 1)) {
        load_b(0);
        publish_b(0);
    }
    for (int step = 0; step < (PB ? 0 : nsteps); ++step) {
        const int t = step % p.T;
        if (!(DBG & 1) || t == 0) __syncthreads();  // the previous step's fragment reads are done; weight max published
        int ea2 = ea;
        if (t == 0 && (!(DBG & 4) || step == 0)) ea2 = stage_a(c_begin + step / p.T, ea);  // (contains a barrier)
        float mmb = 0.f;
#pragma unroll
        for (int w = 0; w < NTH / 64; ++w) mmb = fmaxf(mmb, s_redb[step & 1][w]);
        const int eb2 = tile_exp(mmb, eb);
        if (ea2 + eb2 != ea + eb) {
            const int d = ea2 + eb2 - ea - eb;
#pragma unroll
            for (int i = 0; i < WM; ++i)
#pragma unroll
                for (int k = 0; k < WN; ++k)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[i][k][r] = ldexpf(acc[i][k][r], d);
        }
        ea = ea2;
        eb = eb2;
        const float sb = ldexpf(1.f, eb);
        if constexpr (!(DBG & 1)) {
#pragma unroll
            for (int k = 0; k < BX_IT; ++k) {
                const int idx = tid + k * NTH;
                split_put(s_b + (idx >> 3) * XPn, idx & 7, rb[k], sb);
            }
            __syncthreads();
            if (step + 1 < nsteps) load_b(step + 1);
        }
        const int dy = p.offy[t] - h.oymin, dx = p.offx[t] - h.oxmin;
        const int mc = ml % CW, mr = ml / CW;  // the lane's M row: column mc of tile row mr of its M-tile
        const int col = (h.npar == 1) ? mc + dx : (dx & 1) * h.IXp + mc + (dx >> 1);
        const unsigned char *a_base[WM];
#pragma unroll
        for (int i = 0; i < WM; ++i) {
            const int ty = wm * WM + i;
            a_base[i] = s_a + ((p.smy * (RPM * ty + mr) + dy) * h.IXt + col) * XPn + 16 * hl;
        }
#pragma unroll
        for (int s2 = 0; s2 < ((DBG & 2) ? 0 : 2); ++s2) {
            f16x8 ah[WM], al[WM], al2[WM];
#pragma unroll
            for (int i = 0; i < WM; ++i) {
                ah[i] = *reinterpret_cast<const f16x8 *>(a_base[i] + 32 * s2);
                al[i] = *reinterpret_cast<const f16x8 *>(a_base[i] + 64 + 32 * s2);
                if (NP == 3) al2[i] = *reinterpret_cast<const f16x8 *>(a_base[i] + 128 + 32 * s2);
            }
#pragma unroll
            for (int k = 0; k < WN; ++k) {
                const unsigned char *b0 = s_b + ((wn * WN + k) * 32 + ml) * XPn + 16 * hl + 32 * s2;
                const f16x8 bh = *reinterpret_cast<const f16x8 *>(b0);
                const f16x8 bl = *reinterpret_cast<const f16x8 *>(b0 + 64);
                f16x8 bl2;
                if (NP == 3) bl2 = *reinterpret_cast<const f16x8 *>(b0 + 128);
#pragma unroll
                for (int i = 0; i < WM; ++i) {
                    if (NP == 3) {
                        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al2[i], bh, acc[i][k], 0, 0, 0);
                        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl2, acc[i][k], 0, 0, 0);
                        acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bl, acc[i][k], 0, 0, 0);
                    }
                    acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh, acc[i][k], 0, 0, 0);
                    acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl, acc[i][k], 0, 0, 0);
                    acc[i][k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh, acc[i][k], 0, 0, 0);
                }
            }
        }
        if (!(DBG & 1) && step + 1 < nsteps) publish_b((step + 1) & 1);
    }

    const long long per_img = (long long)p.MH * p.MW;
    const int ue = -(ea + eb);
#pragma unroll
    for (int i = 0; i < WM; ++i) {
        const int Yt = Y0 + RPM * (wm * WM + i);  // first output row of M-tile i
        if (Yt >= p.MH) continue;
#pragma unroll
        for (int k = 0; k < WN; ++k) {
            const int n = n0 + (wn * WN + k) * 32 + ml;
            if (gridDim.z > 1) {
                float *part = p.partial + (long long)blockIdx.z * p.B * per_img * p.n_pad;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = (r & 3) + 8 * (r >> 2) + 4 * hl;
                    const int Y = Yt + m / CW, X = X0 + m % CW;
                    if (X < p.MW && Y < p.MH)
                        part[(b * per_img + (long long)Y * p.MW + X) * p.n_pad + n] = ldexpf(acc[i][k][r], ue);
                }
                continue;
            }
            if (n >= p.n) continue;
            const float bn = p.bias ? p.bias[n] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = (r & 3) + 8 * (r >> 2) + 4 * hl;
                const int Y = Yt + m / CW, X = X0 + m % CW;
                if (X < p.MW && Y < p.MH) put_out(p, b, Y, X, n, ldexpf(acc[i][k][r], ue) + bn);
            }
        }
    }
}

// out[map(m)][n] = bias[n] + Σ_z partial[z][m][n], z in order (deterministic)
__global__ void dconv_splitk_reduce(FwdParams p, int ksplit) {
    const long long M = (long long)p.B * p.MH * p.MW;
    const long long i = (long long)blockIdx.x * NTH + threadIdx.x;
    if (i >= M * p.n) return;
    const long long m = i / p.n;
    const int n = (int)(i - m * p.n);
    float v = 0.f;
    for (int z = 0; z < ksplit; ++z) v += p.partial[((long long)z * M + m) * p.n_pad + n];
    const int per_img = p.MH * p.MW;
    const int b = (int)(m / per_img), rr = (int)(m - (long long)b * per_img);
    const int Y = rr / p.MW, X = rr - Y * p.MW;
    put_out(p, b, Y, X, n, v + (p.bias ? p.bias[n] : 0.f));
}

// ---- weight gradient ------------------------------------------------------------------------------------------------
constexpr int WKP = 64;   // pixels per K step
constexpr int WPS = 68;   // LDS row pitch (floats) of the [pixel][64 channels] tiles

struct WgradParams {
    const float *src;
    int B, Hs, Ws, sp, cin, svec;
    const float *dy;
    int MH, MW, dp, cout, dvec;
    int smy, smx, T;
    int ci_blocks, co_blocks;
    long long pix_per_split;
    float *partial;
    int offy[MAXT], offx[MAXT];
};

__global__ __launch_bounds__(NTH, 2) void dconv_wgrad_kernel(WgradParams p) {
    __shared__ __attribute__((aligned(16))) float lds[2 * WKP * WPS];
    float *s_a = lds, *s_b = lds + WKP * WPS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5, ml = lane & 31;
    int bid = blockIdx.x;
    const int cob = bid % p.co_blocks;
    bid /= p.co_blocks;
    const int cib = bid % p.ci_blocks;
    const int t = bid / p.ci_blocks;
    const int split = blockIdx.y;
    const int per_img = p.MH * p.MW;
    const long long P = (long long)p.B * per_img;
    const long long k0 = (long long)split * p.pix_per_split;
    const long long k1 = min(P, k0 + p.pix_per_split);
    const int ci0 = cib * 64, co0 = cob * 64;
    const int oy = p.offy[t], ox = p.offx[t];
    const int c4 = tid & 15;  // 4-channel group staged by this thread (the same for all of its pixel rows)
    const bool svec = p.svec != 0, dvec = p.dvec != 0;
    f32x4 ra[4], rb[4];
    auto load = [&](long long kb) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const long long m = kb + (tid >> 4) + 16 * k;
            f32x4 va = {0.f, 0.f, 0.f, 0.f}, vb = {0.f, 0.f, 0.f, 0.f};
            if (m < k1) {
                const int b = (int)(m / per_img), r = (int)(m - (long long)b * per_img);
                const int Y = r / p.MW, X = r - (r / p.MW) * p.MW;
                const int ci = ci0 + 4 * c4, co = co0 + 4 * c4;
                const int sy = p.smy * Y + oy, sx = p.smx * X + ox;
                if (ci < p.cin && sy >= 0 && sy < p.Hs && sx >= 0 && sx < p.Ws)
                    va = load4(p.src + (((long long)b * p.Hs + sy) * p.Ws + sx) * p.sp, ci, p.cin, svec);
                if (co < p.cout) vb = load4(p.dy + (((long long)b * p.MH + Y) * p.MW + X) * p.dp, co, p.cout, dvec);
            }
            ra[k] = va;
            rb[k] = vb;
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int pp = (tid >> 4) + 16 * k;
            *reinterpret_cast<f32x4 *>(s_a + pp * WPS + 4 * c4) = ra[k];
            *reinterpret_cast<f32x4 *>(s_b + pp * WPS + 4 * c4) = rb[k];
        }
    };
    const int mt = wave >> 1, nt = wave & 1;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if (k0 < k1) load(k0);
    for (long long kb = k0; kb < k1; kb += WKP) {
        __syncthreads();
        store();
        __syncthreads();
        if (kb + WKP < k1) load(kb + WKP);
        // A[m = ci][k = pixel] from s_a[pixel][ci], B[k = pixel][n = co] from s_b[pixel][co]; lane half = pixel parity
#pragma unroll 8
        for (int s = 0; s < WKP / 2; ++s) {
            const float a = s_a[(2 * s + hl) * WPS + 32 * mt + ml];
            const float b = s_b[(2 * s + hl) * WPS + 32 * nt + ml];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
    }
    const int cin_pad = 64 * p.ci_blocks, cout_pad = 64 * p.co_blocks;
    float *dst = p.partial + ((long long)split * p.T + t) * cin_pad * cout_pad;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int ci = ci0 + 32 * mt + (r & 3) + 8 * (r >> 2) + 4 * hl;
        const int co = co0 + 32 * nt + ml;
        dst[(long long)ci * cout_pad + co] = acc[r];
    }
}

// ---- x3 weight gradient ----------------------------------------------------------------------------------------------
// dconv_wgrad's GEMM (M = input channels, N = output channels, K = pixels) on v_mfma_f32_32x32x16_f16 in the split
// scheme, operands split at staging after a per-K-step (64 pixels) power-of-two scaling of each (as
// dconv_fwd_x3_kernel).  Workgroup tile CIB × COB channels (64 or 128 each), 4 waves in 2 × 2, each wave
// (CIB/64) × (COB/64) 32×32 accumulators.  LDS: per pixel one row of 32-byte chunks, logical chunks [hi of channels
// 16j..16j+15]_j then [lo ...]_j, stored at physical chunk (logical ^ 2·(row & 3)); fragments come from
// ds_read_b64_tr_b16 (4 pixel rows × 16 channels per 16-lane group), and with the XOR the 4 rows × 2 chunks of a
// half-wave's read cover the 64 banks once.
// NP = 3 (x6): a third piece lo2 and the products lo·lo, hi·lo2, lo2·hi too (see dconv_fwd_x3_kernel).  Rows are
// then 6·nch bytes; for nch = 64 (384 B ≡ 128 mod 256) the XOR swizzle is 2·((row >> 1) & 1) instead of 2·(row & 3)
// so that the 4 rows × 64 B of a half-wave's transposed read still cover the 64 banks once.
template <int CIB, int COB, int NP>
__global__ __launch_bounds__(NTH, 2) void dconv_wgrad_x3_kernel(WgradParams p) {
    constexpr int AQ = CIB / 16, BQ = COB / 16;            // fp32 quads per thread per K step
    constexpr int AROW = 2 * NP * CIB, BROW = 2 * NP * COB; // LDS row bytes (hi + lo [+ lo2])
    constexpr int MTW = CIB / 64, NTW = COB / 64;           // accumulator tiles per wave
    __shared__ __attribute__((aligned(16))) unsigned char lds[WKP * (AROW + BROW)];
    __shared__ float s_red[2][2][NTH / 64];
    __shared__ long long s_tab[2][2][WKP];  // per K step: source / output-gradient element offset of each pixel row
    unsigned char *s_a = lds, *s_b = lds + WKP * AROW;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5;
    const int nci = (p.cin + CIB - 1) / CIB, nco = (p.cout + COB - 1) / COB;
    int bid = blockIdx.x;
    const int cob = bid % nco;
    bid /= nco;
    const int cib = bid % nci;
    const int t = bid / nci;
    const int split = blockIdx.y;
    const int per_img = p.MH * p.MW;
    const long long P = (long long)p.B * per_img;
    const long long k0 = (long long)split * p.pix_per_split;
    const long long k1 = min(P, k0 + p.pix_per_split);
    const int ci0 = cib * CIB, co0 = cob * COB;
    const int oy = p.offy[t], ox = p.offx[t];
    const bool svec = p.svec != 0, dvec = p.dvec != 0;
    // Pixel table: wave 0's lane r tracks pixel m = kb + r of the current K step as (b, Y, X), advancing by WKP per
    // step without divisions, and publishes the two element offsets (-1: outside the split / the source image).
    int tb = 0, tY = 0, tX = 0;
    if (wave == 0) {
        const long long m = k0 + lane;
        tb = (int)(m / per_img);
        const int r = (int)(m - (long long)tb * per_img);
        tY = r / p.MW;
        tX = r - tY * p.MW;
    }
    auto table = [&](long long kb, int slot) {  // wave 0 only; pixel of (tb, tY, tX) is kb + lane
        long long ao = -1, dofs = -1;
        if (kb + lane < k1) {
            const int sy = p.smy * tY + oy, sx = p.smx * tX + ox;
            if (sy >= 0 && sy < p.Hs && sx >= 0 && sx < p.Ws) ao = (((long long)tb * p.Hs + sy) * p.Ws + sx) * p.sp;
            dofs = (((long long)tb * p.MH + tY) * p.MW + tX) * p.dp;
        }
        s_tab[slot][0][lane] = ao;
        s_tab[slot][1][lane] = dofs;
        tX += WKP;
        while (tX >= p.MW) {
            tX -= p.MW;
            if (++tY == p.MH) {
                tY = 0;
                ++tb;
            }
        }
    };
    // staging roles: thread -> (pixel row, 4-channel quad); quads per row CIB/4 (A) and COB/4 (B)
    f32x4 ra[AQ], rb[BQ];
    auto load = [&](int slot) {
#pragma unroll
        for (int k = 0; k < AQ; ++k) {
            const int idx = tid + k * NTH, row = idx / (CIB / 4), q4 = idx % (CIB / 4);
            const long long ao = s_tab[slot][0][row];
            const int ci = ci0 + 4 * q4;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (ao >= 0 && ci < p.cin) v = load4(p.src + ao, ci, p.cin, svec);
            ra[k] = v;
        }
#pragma unroll
        for (int k = 0; k < BQ; ++k) {
            const int idx = tid + k * NTH, row = idx / (COB / 4), q4 = idx % (COB / 4);
            const long long dofs = s_tab[slot][1][row];
            const int co = co0 + 4 * q4;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (dofs >= 0 && co < p.cout) v = load4(p.dy + dofs, co, p.cout, dvec);
            rb[k] = v;
        }
    };
    auto publish = [&](int slot) {
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int k = 0; k < AQ; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) ma = fmaxf(ma, fabsf(ra[k][e]));
#pragma unroll
        for (int k = 0; k < BQ; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) mb = fmaxf(mb, fabsf(rb[k][e]));
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) {
            ma = fmaxf(ma, __shfl_xor(ma, s));
            mb = fmaxf(mb, __shfl_xor(mb, s));
        }
        if (lane == 0) {
            s_red[slot][0][wave] = ma;
            s_red[slot][1][wave] = mb;
        }
    };
    // byte offset of (row, channel c (multiple of 4), piece) in an image with NCH channels
    auto off = [](int row, int c, int piece, int nch) {
        const int logical = piece * (nch / 16) + (c >> 4);
        const int sw = (NP == 3 && nch == 64) ? 2 * ((row >> 1) & 1) : 2 * (row & 3);
        return row * 2 * NP * nch + ((logical ^ sw) << 5) + (c & 15) * 2;
    };
    auto put = [&](unsigned char *img, int nch, int row, int c, f32x4 v, float s) {
        f16x4 h, l, l2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float x = v[e] * s;
            h[e] = (_Float16)x;
            const float r = x - (float)h[e];
            l[e] = (_Float16)r;
            if (NP == 3) l2[e] = (_Float16)(r - (float)l[e]);
        }
        *reinterpret_cast<f16x4 *>(img + off(row, c, 0, nch)) = h;
        *reinterpret_cast<f16x4 *>(img + off(row, c, 1, nch)) = l;
        if (NP == 3) *reinterpret_cast<f16x4 *>(img + off(row, c, 2, nch)) = l2;
    };

    const int wm = wave >> 1, wn = wave & 1;
    f32x16 acc[MTW][NTW];
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    int ea = 0, eb = 0;
    // transposed-read lane roles (see wgrad3_kernel): row rq of the 4, channel block 4·(lane & 3) of the 16 of group
    const int i16 = lane & 15, rq = i16 >> 2, grp = (lane >> 4) & 1;
    const int cblk = 16 * grp + 4 * (i16 & 3);  // channel offset within a 32-channel tile

    if (wave == 0) table(k0, 0);
    __syncthreads();
    if (k0 < k1) {
        load(0);
        publish(0);
    }
    for (long long kb = k0; kb < k1; kb += WKP) {
        const int it = (int)((kb - k0) / WKP);
        __syncthreads();
        if (wave == 0 && kb + WKP < k1) table(kb + WKP, (it + 1) & 1);
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int w = 0; w < NTH / 64; ++w) {
            ma = fmaxf(ma, s_red[it & 1][0][w]);
            mb = fmaxf(mb, s_red[it & 1][1][w]);
        }
        const int ea2 = tile_exp(ma, ea), eb2 = tile_exp(mb, eb);
        if (ea2 + eb2 != ea + eb) {
            const int d = ea2 + eb2 - ea - eb;
#pragma unroll
            for (int i = 0; i < MTW; ++i)
#pragma unroll
                for (int j = 0; j < NTW; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[i][j][r] = ldexpf(acc[i][j][r], d);
        }
        ea = ea2;
        eb = eb2;
        const float sa = ldexpf(1.f, ea), sb = ldexpf(1.f, eb);
#pragma unroll
        for (int k = 0; k < AQ; ++k) {
            const int idx = tid + k * NTH;
            put(s_a, CIB, idx / (CIB / 4), 4 * (idx % (CIB / 4)), ra[k], sa);
        }
#pragma unroll
        for (int k = 0; k < BQ; ++k) {
            const int idx = tid + k * NTH;
            put(s_b, COB, idx / (COB / 4), 4 * (idx % (COB / 4)), rb[k], sb);
        }
        __syncthreads();
        if (kb + WKP < k1) load((it + 1) & 1);
#pragma unroll
        for (int kq = 0; kq < WKP / 16; ++kq) {
            const int r0 = 16 * kq + 8 * hl + rq;  // K rows (pixels) r0 and r0 + 4 of this lane's two reads
            f16x8 bh[NTW], bl[NTW], bl2[NTW];
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const int c = 32 * (NTW * wn + j) + cblk;
                bh[j] = cat8(tr_read(s_b, off(r0, c, 0, COB)), tr_read(s_b, off(r0 + 4, c, 0, COB)));
                bl[j] = cat8(tr_read(s_b, off(r0, c, 1, COB)), tr_read(s_b, off(r0 + 4, c, 1, COB)));
                if (NP == 3)
                    bl2[j] = cat8(tr_read(s_b, off(r0, c, 2, COB)), tr_read(s_b, off(r0 + 4, c, 2, COB)));
            }
#pragma unroll
            for (int i = 0; i < MTW; ++i) {
                const int c = 32 * (MTW * wm + i) + cblk;
                const f16x8 ah = cat8(tr_read(s_a, off(r0, c, 0, CIB)), tr_read(s_a, off(r0 + 4, c, 0, CIB)));
                const f16x8 al = cat8(tr_read(s_a, off(r0, c, 1, CIB)), tr_read(s_a, off(r0 + 4, c, 1, CIB)));
                f16x8 al2;
                if (NP == 3) al2 = cat8(tr_read(s_a, off(r0, c, 2, CIB)), tr_read(s_a, off(r0 + 4, c, 2, CIB)));
#pragma unroll
                for (int j = 0; j < NTW; ++j) {
                    if (NP == 3) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al2, bh[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl2[j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bl[j], acc[i][j], 0, 0, 0);
                    }
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[j], acc[i][j], 0, 0, 0);
                }
            }
        }
        if (kb + WKP < k1) publish((it + 1) & 1);
    }
    const int cin_pad = 64 * p.ci_blocks, cout_pad = 64 * p.co_blocks;
    float *dst = p.partial + ((long long)split * p.T + t) * cin_pad * cout_pad;
    const int ml = lane & 31;
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int ci = ci0 + 32 * (MTW * wm + i) + (r & 3) + 8 * (r >> 2) + 4 * hl;
                const int co = co0 + 32 * (NTW * wn + j) + ml;
                if (ci < cin_pad && co < cout_pad)
                    dst[(long long)ci * cout_pad + co] = ldexpf(acc[i][j][r], -(ea + eb));
            }
}

// ---- tap-row weight gradient (split x3 / x6) ----------------------------------------------------------------------------
// dconv_wgrad_x3_kernel re-gathers the 64 source pixels of a K step for every tap (one tap per workgroup) and reloads
// the output gradient for every tap.  Here a workgroup owns one ROW of the kernel (the KT taps (ky, 0..KT-1), which
// share a source row) and a K step is a 64-pixel segment of one output row: the output-gradient segment [64 px][COB]
// and the source row segment covering all KT taps (64 + KT - 1 pixels at stride 1; two column-parity halves of
// 64 + (KT - 1)/2 at stride 2) are staged once per step, and every tap reads its A fragments at its column offset —
// KT× less output-gradient staging and ~KT× less source staging.  Operands in NP f16 pieces with a per-step power-of-
// two scale per operand (dconv_wgrad_x3_kernel's scheme); LDS images and transposed fragment reads as there (any 4
// consecutive rows are conflict-free under the XOR swizzle, so a tap's shifted rows keep that).
struct WrowParams {
    const float *src;
    int B, Hs, Ws, sp, cin, svec;
    const float *dy;
    int MH, MW, dp, cout, dvec;
    int smy, smx, T, KT;  // taps; taps per group = the kernel width (group g = taps g·KT .. g·KT + KT - 1)
    int nseg;             // 64-pixel segments per output row
    long long segs_per_split;
    int HP;               // staged source columns per parity
    int ci_blocks, co_blocks;  // 64-channel units of the partial layout
    float *partial;            // [split][T][64·ci_blocks][64·co_blocks]
    int offy[MAXT], offx[MAXT];
};

constexpr int WSEG = 64;  // output pixels per K step

template <int CIB, int COB, int NP, int KT, int SMX>
__global__ __launch_bounds__(NTH, 1) void dconv_wgrad_rows_kernel(WrowParams p) {
    constexpr int HPM = SMX == 1 ? WSEG + KT - 1 : WSEG + (KT - 1) / 2;  // columns per parity (max)
    constexpr int AROWS = SMX * HPM;
    constexpr int AQ = (AROWS * CIB / 4 + NTH - 1) / NTH, BQ = WSEG * COB / 4 / NTH;
    constexpr int AROW = 2 * NP * CIB;
    constexpr int MTW = CIB / 64, NTW = COB / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char rlds[];
    unsigned char *s_a = rlds, *s_b = rlds + AROWS * AROW;
    __shared__ float s_red[2][2][NTH / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane >> 5;
    const int nci = (p.cin + CIB - 1) / CIB, nco = (p.cout + COB - 1) / COB;
    int bid = blockIdx.x;
    const int cob = bid % nco;
    bid /= nco;
    const int cib = bid % nci;
    const int g = bid / nci;  // kernel row
    const int t0 = g * KT;
    const int ci0 = cib * CIB, co0 = cob * COB;
    const int oy = p.offy[t0], oxmin = p.offx[t0];
    const long long nsegs = (long long)p.B * p.MH * p.nseg;
    const long long q0 = (long long)blockIdx.y * p.segs_per_split;
    const long long q1 = min(nsegs, q0 + p.segs_per_split);
    const bool svec = p.svec != 0, dvec = p.dvec != 0;

    f32x4 ra[AQ], rb[BQ];
    auto load = [&](long long q) {
        const int b = (int)(q / ((long long)p.MH * p.nseg));
        const int r = (int)(q - (long long)b * p.MH * p.nseg);
        const int Y = r / p.nseg, X0 = (r - Y * p.nseg) * WSEG;
        const int sy = p.smy * Y + oy, sx0 = p.smx * X0 + oxmin;
        const bool row_ok = sy >= 0 && sy < p.Hs;
        const float *srow = p.src + ((long long)b * p.Hs + (row_ok ? sy : 0)) * p.Ws * p.sp;
#pragma unroll
        for (int k = 0; k < AQ; ++k) {
            const int idx = tid + k * NTH, row = idx / (CIB / 4), q4 = idx % (CIB / 4);
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (row < AROWS && row_ok) {
                const int par = row / HPM, h = row - par * HPM;
                const int sx = sx0 + h * SMX + par, ci = ci0 + 4 * q4;
                if (h < p.HP && sx >= 0 && sx < p.Ws && ci < p.cin) v = load4(srow + (long long)sx * p.sp, ci, p.cin, svec);
            }
            ra[k] = v;
        }
        const float *drow = p.dy + (((long long)b * p.MH + Y) * p.MW) * p.dp;
#pragma unroll
        for (int k = 0; k < BQ; ++k) {
            const int idx = tid + k * NTH, row = idx / (COB / 4), q4 = idx % (COB / 4);
            const int X = X0 + row, co = co0 + 4 * q4;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (X < p.MW && co < p.cout) v = load4(drow + (long long)X * p.dp, co, p.cout, dvec);
            rb[k] = v;
        }
    };
    auto publish = [&](int slot) {
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int k = 0; k < AQ; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) ma = fmaxf(ma, fabsf(ra[k][e]));
#pragma unroll
        for (int k = 0; k < BQ; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) mb = fmaxf(mb, fabsf(rb[k][e]));
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) {
            ma = fmaxf(ma, __shfl_xor(ma, s));
            mb = fmaxf(mb, __shfl_xor(mb, s));
        }
        if (lane == 0) {
            s_red[slot][0][wave] = ma;
            s_red[slot][1][wave] = mb;
        }
    };
    auto off = [](int row, int c, int piece, int nch) {
        const int logical = piece * (nch / 16) + (c >> 4);
        const int sw = (NP == 3 && nch == 64) ? 2 * ((row >> 1) & 1) : 2 * (row & 3);
        return row * 2 * NP * nch + ((logical ^ sw) << 5) + (c & 15) * 2;
    };
    auto put = [&](unsigned char *img, int nch, int row, int c, f32x4 v, float sc) {
        f16x4 h, l, l2;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float x = v[e] * sc;
            h[e] = (_Float16)x;
            const float r = x - (float)h[e];
            l[e] = (_Float16)r;
            if (NP == 3) l2[e] = (_Float16)(r - (float)l[e]);
        }
        *reinterpret_cast<f16x4 *>(img + off(row, c, 0, nch)) = h;
        *reinterpret_cast<f16x4 *>(img + off(row, c, 1, nch)) = l;
        if (NP == 3) *reinterpret_cast<f16x4 *>(img + off(row, c, 2, nch)) = l2;
    };

    const int wm = wave >> 1, wn = wave & 1;
    f32x16 acc[KT][MTW][NTW];
#pragma unroll
    for (int x = 0; x < KT; ++x)
#pragma unroll
        for (int i = 0; i < MTW; ++i)
#pragma unroll
            for (int j = 0; j < NTW; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[x][i][j][r] = 0.f;
    int ea = 0, eb = 0;
    const int i16 = lane & 15, rq = i16 >> 2, grp = (lane >> 4) & 1;
    const int cblk = 16 * grp + 4 * (i16 & 3);
    int rowoff[KT];  // staged source row of output pixel 0 for each tap
#pragma unroll
    for (int x = 0; x < KT; ++x) {
        const int d = p.offx[t0 + x] - oxmin;
        rowoff[x] = SMX == 1 ? d : (d & 1) * HPM + (d >> 1);
    }

    if (q0 < q1) {
        load(q0);
        publish(0);
    }
    for (long long q = q0; q < q1; ++q) {
        const int it = (int)(q - q0);
        __syncthreads();
        float ma = 0.f, mb = 0.f;
#pragma unroll
        for (int w = 0; w < NTH / 64; ++w) {
            ma = fmaxf(ma, s_red[it & 1][0][w]);
            mb = fmaxf(mb, s_red[it & 1][1][w]);
        }
        const int ea2 = tile_exp(ma, ea), eb2 = tile_exp(mb, eb);
        if (ea2 + eb2 != ea + eb) {
            const int d = ea2 + eb2 - ea - eb;
#pragma unroll
            for (int x = 0; x < KT; ++x)
#pragma unroll
                for (int i = 0; i < MTW; ++i)
#pragma unroll
                    for (int j = 0; j < NTW; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r) acc[x][i][j][r] = ldexpf(acc[x][i][j][r], d);
        }
        ea = ea2;
        eb = eb2;
        const float sa = ldexpf(1.f, ea), sb = ldexpf(1.f, eb);
#pragma unroll
        for (int k = 0; k < AQ; ++k) {
            const int idx = tid + k * NTH, row = idx / (CIB / 4);
            if (row < AROWS) put(s_a, CIB, row, 4 * (idx % (CIB / 4)), ra[k], sa);
        }
#pragma unroll
        for (int k = 0; k < BQ; ++k) {
            const int idx = tid + k * NTH;
            put(s_b, COB, idx / (COB / 4), 4 * (idx % (COB / 4)), rb[k], sb);
        }
        __syncthreads();
        if (q + 1 < q1) load(q + 1);
#pragma unroll
        for (int kq = 0; kq < WSEG / 16; ++kq) {
            const int r0 = 16 * kq + 8 * hl + rq;  // K rows (output pixels) r0 and r0 + 4 of this lane's two reads
            f16x8 bh[NTW], bl[NTW], bl2[NTW];
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const int c = 32 * (NTW * wn + j) + cblk;
                bh[j] = cat8(tr_read(s_b, off(r0, c, 0, COB)), tr_read(s_b, off(r0 + 4, c, 0, COB)));
                bl[j] = cat8(tr_read(s_b, off(r0, c, 1, COB)), tr_read(s_b, off(r0 + 4, c, 1, COB)));
                if (NP == 3)
                    bl2[j] = cat8(tr_read(s_b, off(r0, c, 2, COB)), tr_read(s_b, off(r0 + 4, c, 2, COB)));
            }
#pragma unroll
            for (int x = 0; x < KT; ++x) {
                const int ra0 = rowoff[x] + r0;
#pragma unroll
                for (int i = 0; i < MTW; ++i) {
                    const int c = 32 * (MTW * wm + i) + cblk;
                    const f16x8 ah = cat8(tr_read(s_a, off(ra0, c, 0, CIB)), tr_read(s_a, off(ra0 + 4, c, 0, CIB)));
                    const f16x8 al = cat8(tr_read(s_a, off(ra0, c, 1, CIB)), tr_read(s_a, off(ra0 + 4, c, 1, CIB)));
                    f16x8 al2;
                    if (NP == 3)
                        al2 = cat8(tr_read(s_a, off(ra0, c, 2, CIB)), tr_read(s_a, off(ra0 + 4, c, 2, CIB)));
#pragma unroll
                    for (int j = 0; j < NTW; ++j) {
                        if (NP == 3) {
                            acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al2, bh[j], acc[x][i][j], 0, 0, 0);
                            acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl2[j], acc[x][i][j], 0, 0, 0);
                            acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bl[j], acc[x][i][j], 0, 0, 0);
                        }
                        acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[j], acc[x][i][j], 0, 0, 0);
                        acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[j], acc[x][i][j], 0, 0, 0);
                        acc[x][i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[j], acc[x][i][j], 0, 0, 0);
                    }
                }
            }
        }
        if (q + 1 < q1) publish((it + 1) & 1);
    }
    const int cin_pad = 64 * p.ci_blocks, cout_pad = 64 * p.co_blocks;
    const int ml = lane & 31;
#pragma unroll
    for (int x = 0; x < KT; ++x) {
        float *dst = p.partial + ((long long)blockIdx.y * p.T + t0 + x) * cin_pad * cout_pad;
#pragma unroll
        for (int i = 0; i < MTW; ++i)
#pragma unroll
            for (int j = 0; j < NTW; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int ci = ci0 + 32 * (MTW * wm + i) + (r & 3) + 8 * (r >> 2) + 4 * hl;
                    const int co = co0 + 32 * (NTW * wn + j) + ml;
                    if (ci < cin_pad && co < cout_pad)
                        dst[(long long)ci * cout_pad + co] = ldexpf(acc[x][i][j][r], -(ea + eb));
                }
    }
}

bool aligned16(const void *ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

constexpr int HALO_LDS_2PER_CU = 80 * 1024;  // two workgroups per CU
constexpr int HALO_LDS_MAX = 160 * 1024;

// Which launches take the halo kernels: stride-1 gathers with one tap (the im2col'd first conv, the 1×1 head) or
// with >= 9 taps (3×3, 8×8) on grids whose width the 32-column tiles cover with <= 30 % waste.  Measured at config 3
// (tools/dconv_ab.py, profiles/r3_dconv_ab.txt): the 4×4 stride-2 forward and the 2×2-tap phase classes of its data
// gradient ran slower than the gather kernel (their source window is 4-6× the outputs), and so did the 8×8 layer's
// data gradient on its 38-wide grid (two tiles for 38 columns).
// The 2×2-tap stride-1 form of a 4×4 stride-2 conv over its space-to-depth source / into its depth-to-space output
// (sd: esr_dconv_fwd_sd) stages each source pixel once per 32 virtual channels — 8 real channels × 4 phases — so its
// window fits 8-row tiles at two workgroups per CU; it takes the halo kernel under the same width rule.
bool halo_wanted(int smy, int smx, int T, int MW, bool sd = false) {
    const int covered = 32 * ((MW + 31) / 32);
    if (g_dconv_halo == 2 && (sd || T >= 9) && smy == 1 && smx == 1) return true;
    return smy == 1 && smx == 1 && (T == 1 || T >= 9 || sd) && 10 * (covered - MW) <= 3 * MW;
}


// Tile width of the halo kernel for a launch: 32, 16 (x3 only: 2 rows × 16 columns per M-tile where a 16-column grid
// meets the ≤ 30 % waste rule and a 32-column one does not — fc8's data gradient on the 38-wide grid at config 3:
// 903 -> 651 us, profiles/r3_dconv_cw16_ab.txt), or 0 for the gather kernel.
int halo_cols(int smy, int smx, int T, int MW, bool sd, int np) {
    if (!g_dconv_halo) return 0;
    if (halo_wanted(smy, smx, T, MW, sd)) return 32;
    const int c16 = 16 * ((MW + 15) / 16);
    if (np == 2 && g_dconv_cw16 && smy == 1 && smx == 1 && (T == 1 || T >= 9) && 10 * (c16 - MW) <= 3 * MW)
        return 16;  // (not the 4-tap space-to-depth forms: slower than their gather at MW 38 / 39, r3_dconv_cw16_ab)
    return 0;
}

// Halo tiling of an esr_dconv_fwd launch with `pitch` LDS bytes per staged pixel row (144: fp32 / x3, 208: x6):
// false if the gather kernel has to run it (stride > 2, or a halo that does not fit in LDS even at 2-row tiles).
bool halo_plan(int MH, int MW, int smy, int smx, int T, const int32_t *offy, const int32_t *offx, HaloParams &h,
               int &lds, int pitch = PS * 4, int nbx = NB, int cw = 32, bool pb = false) {
    if (smy < 1 || smy > 2 || smx < 1 || smx > 2 || (cw == 16 && smx != 1)) return false;
    const int rpm = 32 / cw;  // output rows per M-tile
    int ymin = offy[0], ymax = offy[0], xmin = offx[0], xmax = offx[0];
    for (int t = 1; t < T; ++t) {
        ymin = min(ymin, (int)offy[t]); ymax = max(ymax, (int)offy[t]);
        xmin = min(xmin, (int)offx[t]); xmax = max(xmax, (int)offx[t]);
    }
    h.oymin = ymin;
    h.oxmin = xmin;
    h.npar = smx;
    h.IXp = smx == 1 ? cw + (xmax - xmin) : 32 + ((xmax - xmin) >> 1);
    h.IXt = h.npar * h.IXp;
    const int b_bytes = pb ? 2 * nbx * 128 : nbx * pitch;  // pb: two slots of pre-split weight rows
    for (int pass = 0; pass < 2; ++pass) {
        const int budget = pass == 0 ? HALO_LDS_2PER_CU : HALO_LDS_MAX;
        for (int ty = 8; ty >= 2; ty >>= 1) {
            if (ty > 2 && MH <= rpm * ty / 2) continue;  // a shorter tile wastes fewer rows
            const int iy = smy * (rpm * ty - 1) + (ymax - ymin) + 1;
            const int a_bytes = iy * h.IXt * pitch;
            if (a_bytes + b_bytes <= budget) {
                h.TY = ty;
                h.IY = iy;
                h.b_off = a_bytes;
                h.tiles_x = (MW + cw - 1) / cw;
                h.tiles_y = (MH + rpm * ty - 1) / (rpm * ty);
                h.cw = cw;
                lds = a_bytes + b_bytes;
                return true;
            }
        }
    }
    return false;
}

// split-K slices for a halo launch: enough workgroups to fill the chip twice, at least one chunk per slice
int halo_splits(const HaloParams &h, int B, int n_pad, int nck) {
    const long long wgs = (long long)B * h.tiles_x * h.tiles_y * (n_pad / NB);
    if (wgs >= 512 || nck < 2) return 1;
    return (int)min((long long)nck, (512 + wgs - 1) / wgs);
}

// The tap-row weight-gradient kernel's shape for a launch: kernel width KT (the taps must be (ky, kx) ky-major with
// kx consecutive, as the discriminator's convs list them), channel blocks, LDS bytes; false = the per-tap kernel.
struct RowsPlan {
    int KT, CIB, COB, HP, lds;
};
bool rows_plan(int smx, int T, const int32_t *offy, const int32_t *offx, int np, RowsPlan &r) {
    if (smx < 1 || smx > 2) return false;
    int kt = 1;
    while (kt < T && offy[kt] == offy[0]) ++kt;
    if (T % kt) return false;
    for (int t = 0; t < T; ++t)
        if (offy[t] != offy[t - t % kt] || offx[t] != offx[t - t % kt] + t % kt) return false;
    if (kt != 1 && kt != 3 && kt != 4 && kt != 8) return false;
    if (smx == 2 && kt != 4) return false;
    r.KT = kt;
    // accumulators per lane = KT · (CIB/64) · (COB/64) · 16 and staging registers must fit one wave per SIMD
    r.CIB = kt <= 3 ? 128 : 64;
    r.COB = kt == 1 ? 128 : 64;
    r.HP = smx == 1 ? WSEG + kt - 1 : WSEG + (kt - 1) / 2;
    r.lds = smx * r.HP * 2 * np * r.CIB + WSEG * 2 * np * r.COB;
    return r.lds <= HALO_LDS_MAX - 2048;
}

int rows_splits(const RowsPlan &r, int B, int MH, int MW, int cin, int cout, int T) {
    const long long gx = (long long)(T / r.KT) * ((cin + r.CIB - 1) / r.CIB) * ((cout + r.COB - 1) / r.COB);
    const long long nsegs = (long long)B * MH * ((MW + WSEG - 1) / WSEG);
    const long long n = (long long)T * 64 * ((cin + 63) / 64) * 64 * ((cout + 63) / 64);
    long long sp = (512 + gx - 1) / gx;  // ~2 waves of workgroups over 256 CUs (one resident per CU)
    sp = min(sp, nsegs);
    sp = min(sp, max(1LL, (64LL << 20) / n));  // partial buffer <= 64 M floats
    return (int)max(1LL, sp);
}

// allow a kernel the whole LDS as dynamic shared memory (once per instantiation)
template <typename K>
void allow_full_lds(K kernel, bool &done) {
    if (!done) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  HALO_LDS_MAX - 2048);
        done = true;
    }
}

template <int CIB, int COB, int NP, int KT, int SMX>
void launch_rows(const WrowParams &p, dim3 grid, int lds, hipStream_t st) {
    static bool attr = false;
    allow_full_lds(dconv_wgrad_rows_kernel<CIB, COB, NP, KT, SMX>, attr);
    hipLaunchKernelGGL((dconv_wgrad_rows_kernel<CIB, COB, NP, KT, SMX>), grid, dim3(NTH), lds, st, p);
}

template <int NP>
bool launch_rows_np(const WrowParams &p, const RowsPlan &r, dim3 grid, hipStream_t st) {
    if (r.KT == 1) launch_rows<128, 128, NP, 1, 1>(p, grid, r.lds, st);
    else if (r.KT == 3 && p.smx == 1) launch_rows<128, 64, NP, 3, 1>(p, grid, r.lds, st);
    else if (r.KT == 4 && p.smx == 2) launch_rows<64, 64, NP, 4, 2>(p, grid, r.lds, st);
    else if (r.KT == 4 && p.smx == 1) launch_rows<64, 64, NP, 4, 1>(p, grid, r.lds, st);
    else if (r.KT == 8 && p.smx == 1) launch_rows<64, 64, NP, 8, 1>(p, grid, r.lds, st);
    else return false;
    return true;
}


template <int WM, int WN>
void launch_halo_f32(const FwdParams &p, const HaloParams &h, dim3 grid, int lds, hipStream_t st) {
    static bool attr = false;
    allow_full_lds(dconv_fwd_halo_kernel<WM, WN>, attr);
    hipLaunchKernelGGL((dconv_fwd_halo_kernel<WM, WN>), grid, dim3(NTH), lds, st, p, h);
}

template <int WM, int WN, int NP, int NBX = NB, int DBG = 0, int OCC = 2, int CW = 32, bool PB = false>
void launch_halo_x1(const FwdParams &p, const HaloParams &h, dim3 grid, int lds, hipStream_t st) {
    static bool attr = false;
    allow_full_lds(dconv_fwd_halo_x_kernel<WM, WN, NP, NBX, DBG, OCC, CW, PB>, attr);
    hipLaunchKernelGGL((dconv_fwd_halo_x_kernel<WM, WN, NP, NBX, DBG, OCC, CW, PB>), grid, dim3(NTH), lds, st, p, h);
}

// the pre-split-weight (PB) forms of launch_halo_x's x3 choices
template <int WM, int WN, int NBX = NB>
void launch_halo_pb(const FwdParams &p, const HaloParams &h, dim3 grid, int lds, hipStream_t st) {
    if constexpr (NBX == 64) {
        if (h.cw == 16) {
            if (g_dconv_occ3 && lds <= 160 * 1024 / 3)
                return launch_halo_x1<WM, WN, 2, NBX, 0, 3, 16, true>(p, h, grid, lds, st);
            return launch_halo_x1<WM, WN, 2, NBX, 0, 2, 16, true>(p, h, grid, lds, st);
        }
    }
    if constexpr (NBX == 64 && WM == 2) {
        if (g_dconv_occ3 && lds <= 160 * 1024 / 3) return launch_halo_x1<WM, WN, 2, NBX, 0, 3, 32, true>(p, h, grid, lds, st);
    }
    launch_halo_x1<WM, WN, 2, NBX, 0, 2, 32, true>(p, h, grid, lds, st);
}

template <int WM, int WN, int NP, int NBX = NB>
void launch_halo_x(const FwdParams &p, const HaloParams &h, dim3 grid, int lds, hipStream_t st) {
    if constexpr (NP == 2 && NBX == 64) {
        if (h.cw == 16) {  // 16-column tiles (halo_cols)
            if (g_dconv_occ3 && lds <= 160 * 1024 / 3)
                return launch_halo_x1<WM, WN, NP, NBX, 0, 3, 16>(p, h, grid, lds, st);
            return launch_halo_x1<WM, WN, NP, NBX, 0, 2, 16>(p, h, grid, lds, st);
        }
    }
#ifdef ESR_X3_EXPERIMENTS  // ablations (garbage outputs): ESR_HALO_DBG = 1 / 2 / 4 / combinations (the DBG bits)
    static const int dbg = getenv("ESR_HALO_DBG") ? atoi(getenv("ESR_HALO_DBG")) : 0;
    if (NP == 2 && WM == 2) {
        switch (dbg) {
        case 1: return launch_halo_x1<WM, WN, NP, NBX, 1>(p, h, grid, lds, st);
        case 2: return launch_halo_x1<WM, WN, NP, NBX, 2>(p, h, grid, lds, st);
        case 3: return launch_halo_x1<WM, WN, NP, NBX, 3>(p, h, grid, lds, st);
        case 4: return launch_halo_x1<WM, WN, NP, NBX, 4>(p, h, grid, lds, st);
        case 5: return launch_halo_x1<WM, WN, NP, NBX, 5>(p, h, grid, lds, st);
        case 6: return launch_halo_x1<WM, WN, NP, NBX, 6>(p, h, grid, lds, st);
        default: break;
        }
    }
#endif
    // three workgroups per CU where the window + weight slab fit a third of the LDS (the space-to-depth forms at
    // 8-row tiles: 52 KB) and the kernel a third of the VGPRs (profiles/r3_dconv_occ3_ab.txt)
    if constexpr (NP == 2 && NBX == 64 && WM == 2) {
        if (g_dconv_occ3 && lds <= 160 * 1024 / 3) return launch_halo_x1<WM, WN, NP, NBX, 0, 3>(p, h, grid, lds, st);
    }
    launch_halo_x1<WM, WN, NP, NBX, 0>(p, h, grid, lds, st);
}

}  // namespace



// ---- pre-split x3 weights (esr_dconv_presplit) -------------------------------------------------------------------------
constexpr int PS_BLOCKS = 512;  // partial-max blocks

__global__ __launch_bounds__(NTH) void presplit_amax_kernel(const float *w, long long n, float *partial) {
    __shared__ float red[NTH / 64];
    float m = 0.f;
    for (long long i = (long long)blockIdx.x * NTH + threadIdx.x; i < n; i += (long long)gridDim.x * NTH)
        m = fmaxf(m, fabsf(w[i]));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float mm = 0.f;
#pragma unroll
        for (int k = 0; k < NTH / 64; ++k) mm = fmaxf(mm, red[k]);
        partial[blockIdx.x] = mm;
    }
}

// One 16-byte output slot per thread: row r = (t, j, n), physical slot p holds logical slot l = p ^ ((n >> 1) & 7) =
// piece·4 + k: channels 8k..8k+7 of the row, hi (piece 0) or lo (piece 1) of w·2^E (include/esr_amd.h w_split).
__global__ __launch_bounds__(NTH) void presplit_apply_kernel(const float *wp, long long rows, int n_pad,
                                                             const float *partial, int nparts, _Float16 *out,
                                                             int32_t *wexp) {
    __shared__ float s_e;
    if (threadIdx.x < 64) {  // the tensor's max |w| from the partials (every block, same order: same result)
        float m = 0.f;
        for (int i = threadIdx.x; i < nparts; i += 64) m = fmaxf(m, partial[i]);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        if (threadIdx.x == 0) {
            int e = 0;
            if (m > 0.f) (void)frexpf(m, &e);  // m = f·2^e, f in [0.5, 1): E = 15 - e puts m·2^E in [2^14, 2^15)
            const int E = m > 0.f ? 15 - e : 0;
            s_e = (float)E;
            if (blockIdx.x == 0) *wexp = E;
        }
    }
    __syncthreads();
    const float sc = ldexpf(1.f, (int)s_e);
    const long long q = (long long)blockIdx.x * NTH + threadIdx.x;
    if (q >= rows * 8) return;
    const long long r = q >> 3;
    const int n = (int)(r % n_pad), l = (int)(q & 7) ^ ((n >> 1) & 7), k = l & 3;
    const f32x4 a = *reinterpret_cast<const f32x4 *>(wp + r * 32 + 8 * k);
    const f32x4 b = *reinterpret_cast<const f32x4 *>(wp + r * 32 + 8 * k + 4);
    f16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float x = (e < 4 ? a[e] : b[e - 4]) * sc;
        const _Float16 hi = (_Float16)x;
        v[e] = (l >> 2) ? (_Float16)(x - (float)hi) : hi;
    }
    *reinterpret_cast<f16x8 *>(out + q * 8) = v;
}

// Per-call precision of the discriminator convs (include/esr_amd.h `prec`): 0 = exact fp32, 1 = x3 (128-wide N tiles
// where the grid allows), 2 = x3 with 64-wide N tiles only, 3 = x6.  np = f16 pieces per operand value (0: fp32),
// nb = widest N tile.
struct DPrec {
    int np, nb;
};
bool decode_prec(int32_t prec, DPrec &d) {
    if (prec < 0 || prec > 3) return false;
    d.np = prec == 0 ? 0 : prec == 3 ? 3 : 2;
    d.nb = prec == 2 ? 64 : 128;
    return true;
}

extern "C" int esr_dconv_fwd_sd(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t kc,
                                const float *w_packed, int32_t nck, int32_t n_pad, const float *bias, float *out,
                                int32_t Ho, int32_t Wo, int32_t out_pitch, int32_t n, int32_t MH, int32_t MW,
                                int32_t omy, int32_t oay, int32_t omx, int32_t oax, int32_t smy, int32_t smx, int32_t T,
                                const int32_t *offy, const int32_t *offx, int32_t ksplit, float *partial, int32_t s2d_c,
                                int32_t s2d_pad, int32_t d2s_c, int32_t d2s_pad, int32_t prec, const void *w_split,
                                const int32_t *w_exp, esr_stream_t stream) {
    DPrec dp;
    if (!src || !w_packed || !out || !offy || !offx || !decode_prec(prec, dp)) return ESR_EINVAL;
    if ((w_split == nullptr) != (w_exp == nullptr) || (w_split && ((uintptr_t)w_split & 15))) return ESR_EINVAL;
    if (ksplit < 1 || (ksplit > 1 && (!partial || ksplit > T * nck))) return ESR_EINVAL;
    if (s2d_c < 0 || d2s_c < 0 || s2d_pad < 0 || d2s_pad < 0) return ESR_EINVAL;
    const int src_c = s2d_c ? s2d_c : kc, out_c = d2s_c ? d2s_c : n;  // real channels per source / output pixel
    if (B <= 0 || Hs <= 0 || Ws <= 0 || kc <= 0 || src_pitch < src_c || n <= 0 || out_pitch < out_c || MH <= 0 ||
        MW <= 0)
        return ESR_EINVAL;
    if (T <= 0 || T > ESR_DCONV_MAX_TAPS || nck != (kc + KC - 1) / KC || n_pad % NB || n_pad < n) return ESR_EINVAL;
    if (!aligned16(w_packed)) return ESR_EINVAL;
    if (s2d_c && (s2d_c % 4 || kc != 4 * s2d_c)) return ESR_EINVAL;
    if (d2s_c) {  // every grid point maps to at least one real pixel; the bias would be per virtual channel
        if (n != 4 * d2s_c || bias || omy != 1 || omx != 1 || oay || oax) return ESR_EINVAL;
        if (2 * (MH - 1) - d2s_pad >= Ho || 2 * (MW - 1) - d2s_pad >= Wo) return ESR_EINVAL;
    } else if (oay < 0 || oax < 0 || omy * (MH - 1) + oay >= Ho || omx * (MW - 1) + oax >= Wo) {
        return ESR_EINVAL;  // every output pixel the grid writes must lie inside the output tensor
    }
    const bool sd = s2d_c || d2s_c;
    FwdParams p;
    p.s2c = s2d_c; p.s2pad = s2d_pad; p.d2c = d2s_c; p.d2pad = d2s_pad;
    p.s2g = s2d_c % 32 == 0 ? 32 : s2d_c;  // the channel grouping of the space-to-depth views (include/esr_amd.h)
    p.d2g = d2s_c % 32 == 0 ? 32 : d2s_c;
    p.s2sh = p.d2sh = -1;
    for (int e = 0; e < 31; ++e) {
        if (p.s2g == (1 << e)) p.s2sh = e;
        if (p.d2g == (1 << e)) p.d2sh = e;
    }
    p.src = src; p.B = B; p.Hs = Hs; p.Ws = Ws; p.sp = src_pitch; p.kc = kc;
    p.vec = (src_pitch % 4 == 0 && aligned16(src)) ? 1 : 0;
    p.w = w_packed; p.nck = nck; p.n_pad = n_pad; p.bias = bias;
    p.out = out; p.Ho = Ho; p.Wo = Wo; p.op = out_pitch; p.n = n;
    p.MH = MH; p.MW = MW; p.omy = omy; p.oay = oay; p.omx = omx; p.oax = oax; p.smy = smy; p.smx = smx;
    p.T = T;
    for (int t = 0; t < T; ++t) { p.offy[t] = offy[t]; p.offx[t] = offx[t]; }
    p.partial = partial;
    p.wsx = static_cast<const unsigned char *>(w_split);
    p.wexp = w_exp;
    const long long M = (long long)B * MH * MW;
    const long long gx = (M + MT - 1) / MT;
    if (M + MT >= 0x7fffffffLL) return ESR_EINVAL;  // the kernels index output pixels in 32 bits
    HaloParams h;
    int lds = 0;
    const int np = dp.np;
    const bool pb = np == 2 && w_split != nullptr;  // x3 halo launches take the pre-split weights when given
    const int cwh = halo_cols(smy, smx, T, MW, sd, np);
    if (cwh && halo_plan(MH, MW, smy, smx, T, offy, offx, h, lds, np == 3 ? XPitch<3>::v : PS * 4, NB, cwh, pb)) {
        if (ksplit > nck) return ESR_EINVAL;  // the halo kernels split the channel chunks
        const long long hx = (long long)B * h.tiles_x * h.tiles_y;
        if (hx > 0x7fffffff) return ESR_EINVAL;
        const dim3 hgrid((unsigned)hx, (unsigned)(n_pad / NB), (unsigned)ksplit), block(NTH);
        const hipStream_t st = (hipStream_t)stream;
        if (np == 0) {
            if (h.TY == 8) launch_halo_f32<2, 2>(p, h, hgrid, lds, st);
            else if (h.TY == 4) launch_halo_f32<1, 2>(p, h, hgrid, lds, st);
            else launch_halo_f32<1, 1>(p, h, hgrid, lds, st);
        } else if (np == 2) {
            // 128-channel N tiles where the plan keeps 8-row tiles under the two-per-CU budget and the grid still
            // has >= 512 workgroups without a split (profiles/r3_dconv_nb128_ab.txt)
            HaloParams h2;
            int lds2 = 0;
            if (h.cw == 32 && dp.nb != 64 && ksplit == 1 && n_pad % 128 == 0 && h.TY == 8 && hx * (n_pad / 128) >= 512 &&
                halo_plan(MH, MW, smy, smx, T, offy, offx, h2, lds2, PS * 4, 128, 32, pb) && h2.TY == 8 &&
                lds2 <= HALO_LDS_2PER_CU) {
                const dim3 g2((unsigned)hx, (unsigned)(n_pad / 128), 1);
                if (pb) launch_halo_pb<2, 4, 128>(p, h2, g2, lds2, st);
                else launch_halo_x<2, 4, 2, 128>(p, h2, g2, lds2, st);
            } else if (pb) {
                if (h.TY == 8) launch_halo_pb<2, 2>(p, h, hgrid, lds, st);
                else if (h.TY == 4) launch_halo_pb<1, 2>(p, h, hgrid, lds, st);
                else launch_halo_pb<1, 1>(p, h, hgrid, lds, st);
            } else if (h.TY == 8) launch_halo_x<2, 2, 2>(p, h, hgrid, lds, st);
            else if (h.TY == 4) launch_halo_x<1, 2, 2>(p, h, hgrid, lds, st);
            else launch_halo_x<1, 1, 2>(p, h, hgrid, lds, st);
        } else {
            if (h.TY == 8) launch_halo_x<2, 2, 3>(p, h, hgrid, lds, st);
            else if (h.TY == 4) launch_halo_x<1, 2, 3>(p, h, hgrid, lds, st);
            else launch_halo_x<1, 1, 3>(p, h, hgrid, lds, st);
        }
        if (ksplit > 1)
            hipLaunchKernelGGL(dconv_splitk_reduce, dim3((unsigned)((M * n + NTH - 1) / NTH)), block, 0, st, p,
                               ksplit);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    const dim3 grid((unsigned)gx, (unsigned)((n + NB - 1) / NB)), block(NTH);
    // 128-channel N tiles only where the grid still fills the chip (the A tile then feeds twice the MFMAs)
    const bool wide = n_pad % 128 == 0 && dp.nb != 64 && gx * (n_pad / 128) * ksplit >= 512;
    const dim3 g128((unsigned)gx, (unsigned)(n_pad / 128), (unsigned)ksplit);
    const dim3 g64((unsigned)gx, (unsigned)(n_pad / 64), (unsigned)ksplit);
    const hipStream_t hst = (hipStream_t)stream;
    if (np == 3 && wide)
        hipLaunchKernelGGL((dconv_fwd_x3_kernel<128, 3>), g128, block, 0, hst, p);
    else if (np == 3)
        hipLaunchKernelGGL((dconv_fwd_x3_kernel<64, 3>), g64, block, 0, hst, p);
    else if (np == 2 && wide)
        hipLaunchKernelGGL((dconv_fwd_x3_kernel<128, 2>), g128, block, 0, hst, p);
    else if (np == 2)
        hipLaunchKernelGGL((dconv_fwd_x3_kernel<64, 2>), g64, block, 0, hst, p);
    else
        hipLaunchKernelGGL(dconv_fwd_kernel, grid, block, 0, (hipStream_t)stream, p);
    if (ksplit > 1)
        hipLaunchKernelGGL(dconv_splitk_reduce, dim3((unsigned)((M * n + NTH - 1) / NTH)), block, 0,
                           (hipStream_t)stream, p, ksplit);
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

extern "C" int esr_dconv_fwd_sk(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t kc,
                                const float *w_packed, int32_t nck, int32_t n_pad, const float *bias, float *out,
                                int32_t Ho, int32_t Wo, int32_t out_pitch, int32_t n, int32_t MH, int32_t MW,
                                int32_t omy, int32_t oay, int32_t omx, int32_t oax, int32_t smy, int32_t smx, int32_t T,
                                const int32_t *offy, const int32_t *offx, int32_t ksplit, float *partial,
                                int32_t prec, esr_stream_t stream) {
    return esr_dconv_fwd_sd(src, B, Hs, Ws, src_pitch, kc, w_packed, nck, n_pad, bias, out, Ho, Wo, out_pitch, n, MH,
                            MW, omy, oay, omx, oax, smy, smx, T, offy, offx, ksplit, partial, 0, 0, 0, 0, prec, nullptr,
                            nullptr, stream);
}

extern "C" int esr_dconv_fwd(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t kc,
                             const float *w_packed, int32_t nck, int32_t n_pad, const float *bias, float *out,
                             int32_t Ho, int32_t Wo, int32_t out_pitch, int32_t n, int32_t MH, int32_t MW, int32_t omy,
                             int32_t oay, int32_t omx, int32_t oax, int32_t smy, int32_t smx, int32_t T,
                             const int32_t *offy, const int32_t *offx, int32_t prec, esr_stream_t stream) {
    return esr_dconv_fwd_sk(src, B, Hs, Ws, src_pitch, kc, w_packed, nck, n_pad, bias, out, Ho, Wo, out_pitch, n, MH,
                            MW, omy, oay, omx, oax, smy, smx, T, offy, offx, 1, nullptr, prec, stream);
}

extern "C" int esr_dconv_fwd_splits_sd(int32_t B, int32_t MH, int32_t MW, int32_t n, int32_t kc, int32_t smy,
                                       int32_t smx, int32_t T, const int32_t *offy, const int32_t *offx, int32_t sd,
                                       int32_t prec) {
    DPrec dp;
    if (B <= 0 || MH <= 0 || MW <= 0 || n <= 0 || kc <= 0 || T <= 0 || T > ESR_DCONV_MAX_TAPS || !offy || !offx ||
        !decode_prec(prec, dp))
        return ESR_EINVAL;
    const int nck = (kc + KC - 1) / KC, n_pad = NB * ((n + NB - 1) / NB);
    HaloParams h;
    int lds = 0;
    const int np = dp.np;
    const int cwh = halo_cols(smy, smx, T, MW, sd != 0, np);
    if (cwh && halo_plan(MH, MW, smy, smx, T, offy, offx, h, lds, np == 3 ? XPitch<3>::v : PS * 4, NB, cwh))
        return halo_splits(h, B, n_pad, nck);
    if (!np) return 1;
    // x3 gather kernel: ~512 workgroups, at least 8 K steps per slice, for launches that would fill few CUs
    const long long wgs = ((long long)B * MH * MW + MT - 1) / MT * (n_pad / NB);
    const int nsteps = T * nck;
    if (wgs >= 512 || nsteps < 16) return 1;
    return (int)max(1LL, min((512 + wgs - 1) / wgs, (long long)(nsteps / 8)));
}

extern "C" int esr_dconv_uses_halo(int32_t smy, int32_t smx, int32_t T, int32_t MW, int32_t sd, int32_t prec) {
    DPrec dp;
    if (T <= 0 || T > ESR_DCONV_MAX_TAPS || MW <= 0 || !decode_prec(prec, dp)) return ESR_EINVAL;
    return halo_cols(smy, smx, T, MW, sd != 0, dp.np) ? 1 : 0;
}

extern "C" int esr_dconv_fwd_splits(int32_t B, int32_t MH, int32_t MW, int32_t n, int32_t kc, int32_t smy,
                                    int32_t smx, int32_t T, const int32_t *offy, const int32_t *offx, int32_t prec) {
    return esr_dconv_fwd_splits_sd(B, MH, MW, n, kc, smy, smx, T, offy, offx, 0, prec);
}

extern "C" int esr_dconv_wgrad_splits(int32_t B, int32_t MH, int32_t MW, int32_t cin, int32_t cout, int32_t smy,
                                     int32_t smx, int32_t T, const int32_t *offy, const int32_t *offx,
                                     int32_t prec) {
    DPrec dp;
    if (B <= 0 || MH <= 0 || MW <= 0 || cin <= 0 || cout <= 0 || T <= 0 || T > ESR_DCONV_MAX_TAPS || !offy || !offx ||
        !decode_prec(prec, dp))
        return ESR_EINVAL;
    (void)smy;
    const int cin_pad = 64 * ((cin + 63) / 64), cout_pad = 64 * ((cout + 63) / 64);
    const long long n = (long long)T * cin_pad * cout_pad, P = (long long)B * MH * MW;
    const long long pmax = max(1LL, (64LL << 20) / n);
    RowsPlan rp;
    if (dp.np && g_dconv_rows != 0 && rows_plan(smx, T, offy, offx, dp.np, rp))
        return rows_splits(rp, B, MH, MW, cin, cout, T);
    if (dp.np) {  // per-tap split kernel: 128-channel blocks where the padded widths allow, ~2 workgroups per CU
        const int cib = cin_pad % 128 == 0 ? 128 : 64, cob = cout_pad % 128 == 0 ? 128 : 64;
        const long long tiles = (long long)T * (cin_pad / cib) * (cout_pad / cob);
        return (int)max(1LL, min(min((512 + tiles - 1) / tiles, (P + 255) / 256), pmax));
    }
    const long long tiles = (long long)T * (cin_pad / 64) * (cout_pad / 64);  // fp32: ~4 workgroups per CU
    return (int)max(1LL, min(min((1024 + tiles - 1) / tiles, (P + 255) / 256), pmax));
}

extern "C" int esr_dconv_wgrad(const float *src, int32_t B, int32_t Hs, int32_t Ws, int32_t src_pitch, int32_t cin,
                               const float *dy, int32_t MH, int32_t MW, int32_t dy_pitch, int32_t cout, int32_t smy,
                               int32_t smx, int32_t T, const int32_t *offy, const int32_t *offx, int32_t splits,
                               float *partial, int32_t prec, esr_stream_t stream) {
    DPrec dp;
    if (!src || !dy || !partial || !offy || !offx || !decode_prec(prec, dp)) return ESR_EINVAL;
    if (B <= 0 || Hs <= 0 || Ws <= 0 || cin <= 0 || src_pitch < cin || MH <= 0 || MW <= 0 || cout <= 0 ||
        dy_pitch < cout || T <= 0 || T > ESR_DCONV_MAX_TAPS || splits <= 0)
        return ESR_EINVAL;
    WgradParams p;
    p.src = src; p.B = B; p.Hs = Hs; p.Ws = Ws; p.sp = src_pitch; p.cin = cin;
    p.svec = (src_pitch % 4 == 0 && aligned16(src)) ? 1 : 0;
    p.dy = dy; p.MH = MH; p.MW = MW; p.dp = dy_pitch; p.cout = cout;
    p.dvec = (dy_pitch % 4 == 0 && aligned16(dy)) ? 1 : 0;
    p.smy = smy; p.smx = smx; p.T = T;
    p.ci_blocks = (cin + 63) / 64;
    p.co_blocks = (cout + 63) / 64;
    const long long P = (long long)B * MH * MW;
    p.pix_per_split = ((P + splits - 1) / splits + WKP - 1) / WKP * WKP;
    p.partial = partial;
    for (int t = 0; t < T; ++t) { p.offy[t] = offy[t]; p.offx[t] = offx[t]; }
    RowsPlan rp;
    if (dp.np && g_dconv_rows != 0 && rows_plan(smx, T, offy, offx, dp.np, rp)) {
        WrowParams q;
        q.src = src; q.B = B; q.Hs = Hs; q.Ws = Ws; q.sp = src_pitch; q.cin = cin; q.svec = p.svec;
        q.dy = dy; q.MH = MH; q.MW = MW; q.dp = dy_pitch; q.cout = cout; q.dvec = p.dvec;
        q.smy = smy; q.smx = smx; q.T = T; q.KT = rp.KT;
        q.nseg = (MW + WSEG - 1) / WSEG;
        const long long nsegs = (long long)B * MH * q.nseg;
        q.segs_per_split = (nsegs + splits - 1) / splits;
        q.HP = rp.HP;
        q.ci_blocks = p.ci_blocks; q.co_blocks = p.co_blocks;
        q.partial = partial;
        for (int t = 0; t < T; ++t) { q.offy[t] = offy[t]; q.offx[t] = offx[t]; }
        const long long gx = (long long)(T / rp.KT) * ((cin + rp.CIB - 1) / rp.CIB) * ((cout + rp.COB - 1) / rp.COB);
        const dim3 grid((unsigned)gx, (unsigned)splits);
        const bool ok = dp.np == 3 ? launch_rows_np<3>(q, rp, grid, (hipStream_t)stream)
                                        : launch_rows_np<2>(q, rp, grid, (hipStream_t)stream);
        if (!ok) return ESR_EINVAL;
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if (dp.np) {  // x3 / x6: 128-channel blocks where the padded width is a multiple of 128
        const int cib = (64 * p.ci_blocks) % 128 == 0 ? 128 : 64, cob = (64 * p.co_blocks) % 128 == 0 ? 128 : 64;
        const long long gx = (long long)T * ((cin + cib - 1) / cib) * ((cout + cob - 1) / cob);
        const dim3 grid((unsigned)gx, (unsigned)splits), block(NTH);
        const hipStream_t st = (hipStream_t)stream;
        if (dp.np == 3) {
            if (cib == 128 && cob == 128) hipLaunchKernelGGL((dconv_wgrad_x3_kernel<128, 128, 3>), grid, block, 0, st, p);
            else if (cib == 128) hipLaunchKernelGGL((dconv_wgrad_x3_kernel<128, 64, 3>), grid, block, 0, st, p);
            else if (cob == 128) hipLaunchKernelGGL((dconv_wgrad_x3_kernel<64, 128, 3>), grid, block, 0, st, p);
            else hipLaunchKernelGGL((dconv_wgrad_x3_kernel<64, 64, 3>), grid, block, 0, st, p);
        } else if (cib == 128 && cob == 128) hipLaunchKernelGGL((dconv_wgrad_x3_kernel<128, 128, 2>), grid, block, 0, st, p);
        else if (cib == 128) hipLaunchKernelGGL((dconv_wgrad_x3_kernel<128, 64, 2>), grid, block, 0, st, p);
        else if (cob == 128) hipLaunchKernelGGL((dconv_wgrad_x3_kernel<64, 128, 2>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((dconv_wgrad_x3_kernel<64, 64, 2>), grid, block, 0, st, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    const long long gx = (long long)T * p.ci_blocks * p.co_blocks;
    const dim3 grid((unsigned)gx, (unsigned)splits), block(NTH);
    hipLaunchKernelGGL(dconv_wgrad_kernel, grid, block, 0, (hipStream_t)stream, p);
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

extern "C" int esr_dconv_presplit(const float *w_packed, int64_t rows, int32_t n_pad, float *scratch, void *w_split,
                                  int32_t *w_exp, esr_stream_t stream) {
    if (!w_packed || !scratch || !w_split || !w_exp || rows <= 0 || n_pad <= 0 || n_pad % NB || rows % n_pad ||
        ((uintptr_t)w_packed & 15) || ((uintptr_t)w_split & 15))
        return ESR_EINVAL;
    const hipStream_t st = (hipStream_t)stream;
    const long long n = rows * 32;
    const int nb = (int)min((long long)PS_BLOCKS, (n + NTH - 1) / NTH);
    hipLaunchKernelGGL(presplit_amax_kernel, dim3(nb), dim3(NTH), 0, st, w_packed, n, scratch);
    hipLaunchKernelGGL(presplit_apply_kernel, dim3((unsigned)((rows * 8 + NTH - 1) / NTH)), dim3(NTH), 0, st, w_packed,
                       (long long)rows, n_pad, (const float *)scratch, nb, static_cast<_Float16 *>(w_split), w_exp);
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

// ---- the first conv's tap gather (HipConv2d._im2col: 3 channels × 9 taps -> one 32-wide K step) ------------------------
namespace {

// out[b][y][x][t·C + c] = x[b][y + ky - p][x + kx - p][c] (zero outside), t = ky·k + kx < k², zero-filled to 32
// channels: one thread per output pixel, its 128-B record written as 8 16-B stores
__global__ __launch_bounds__(256) void im2col32_kernel(const float *__restrict__ x, int B, int H, int W, int C, int k,
                                                       int p, int Ho, int Wo, float *__restrict__ out) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)B * Ho * Wo) return;
    const int xo = idx % Wo;
    const int yo = (idx / Wo) % Ho;
    const long long b = idx / ((long long)Wo * Ho);
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = 0.f;
    for (int t = 0; t < k * k; ++t) {
        const int yy = yo + t / k - p, xx = xo + t % k - p;
        if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
        const float *src = x + ((b * H + yy) * W + xx) * C;
        for (int c = 0; c < C; ++c) v[t * C + c] = src[c];
    }
    float4 *o = reinterpret_cast<float4 *>(out + idx * 32);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
}

// its adjoint: gx[b][y][x][c] = Σ_t gc[b][y - ky + p][x - kx + p][t·C + c] over the outputs in range, added from 0 in
// tap order (as the k² shifted in-place adds of the PyTorch form did): one thread per input pixel
__global__ __launch_bounds__(256) void col2im32_kernel(const float *__restrict__ gc, int B, int Ho, int Wo, int k, int p,
                                                       int H, int W, int C, float *__restrict__ gx) {
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)B * H * W) return;
    const int xx = idx % W;
    const int yy = (idx / W) % H;
    const long long b = idx / ((long long)W * H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < k * k; ++t) {
        const int yo = yy - t / k + p, xo = xx - t % k + p;
        if (yo < 0 || yo >= Ho || xo < 0 || xo >= Wo) continue;
        const float *src = gc + ((b * Ho + yo) * Wo + xo) * 32 + t * C;
        for (int c = 0; c < C; ++c) acc[c] += src[c];
    }
    float *o = gx + idx * C;
    for (int c = 0; c < C; ++c) o[c] = acc[c];
}

}  // namespace

extern "C" int esr_dconv_im2col(const float *x, int32_t B, int32_t H, int32_t W, int32_t C, int32_t k, int32_t p,
                                float *out, esr_stream_t stream) {
    if (!x || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0 || k <= 0 || p < 0 || k * k * C > 32 ||
        (reinterpret_cast<uintptr_t>(out) & 15))
        return ESR_EINVAL;
    const int Ho = H + 2 * p - k + 1, Wo = W + 2 * p - k + 1;
    if (Ho <= 0 || Wo <= 0) return ESR_EINVAL;
    const long long n = (long long)B * Ho * Wo;
    hipLaunchKernelGGL(im2col32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, B, H,
                       W, C, k, p, Ho, Wo, out);
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

extern "C" int esr_dconv_col2im(const float *gc, int32_t B, int32_t H, int32_t W, int32_t C, int32_t k, int32_t p,
                                float *gx, esr_stream_t stream) {
    if (!gc || !gx || B <= 0 || H <= 0 || W <= 0 || C <= 0 || C > 8 || k <= 0 || p < 0 || k * k * C > 32)
        return ESR_EINVAL;
    const int Ho = H + 2 * p - k + 1, Wo = W + 2 * p - k + 1;
    if (Ho <= 0 || Wo <= 0) return ESR_EINVAL;
    const long long n = (long long)B * H * W;
    hipLaunchKernelGGL(col2im32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, gc, B,
                       Ho, Wo, k, p, H, W, C, gx);
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}
