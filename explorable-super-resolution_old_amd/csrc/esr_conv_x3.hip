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
// ds_write) into one of two LDS stages while the MFMAs consume the other stage.  LDS is laid out [in0|in1|w0|w1] and
// the chunk loop is unrolled by two, so every fragment address is a per-lane register computed once per workgroup
// plus an immediate offset (no address arithmetic per tap); DMA source offsets are also computed once.  Fragments
// of tap t+1 are read while tap t's MFMAs run, and the MFMAs are issued product-major over the independent
// accumulators.  Records are 64 B (4 × 16-B slots)
// with the slot index XOR-swizzled by (record>>2)&3, applied on the DMA source address (the DMA destination is
// lane-linear), so the 16 lanes of every ds_read_b128 group hit 16 distinct slots.  Out-of-range halo pixels and
// the channels past cin of a partial chunk are fetched from a zero page.
// Epilogue: accumulators are re-staged through LDS as fp32 [pixel][channel]; each thread finishes 8-channel groups:
// 1/w_scale, bias, LeakyReLU, residuals (split inputs), split + 16-byte stores, or fp32 planar stores for CEM.
#include <hip/hip_runtime.h>
#include "esr_amd.h"
#include "esr_x3c.h"
#include "esr_knobs.h"

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
#ifndef X3_PF
#define X3_PF 2   // fragment prefetch distance (taps) of the classic kernel
#endif

__device__ __attribute__((aligned(16))) unsigned char g_zero_page[64];

struct X3Params {
    const unsigned char *in;
    int B, H, W, in_cp, cin;
    const unsigned char *w;
    const float *bias;
    float w_scale_inv;
    int cout;
    int tap_y0, tap_x0, tiles_x, tiles_y;
    int xcd_map;  // 1: blockIdx -> tile grouped per XCD (xcd_tile)
    int *overflow;
    esr_conv_out o;
};

__device__ __forceinline__ float lrelu(float v) { return v > 0.f ? v : 0.2f * v; }

// Epilogue after 1/w_scale and bias (include/esr_amd.h esr_conv_out): LeakyReLU (lrelu 1), residuals; lrelu 3 = the
// LeakyReLU backward through the saved split activation r2 (data-gradient convs of the x3 backward; r2 not added).
__device__ __forceinline__ float epi(const esr_conv_out &o, float v, float r1, float r2) {
    if (o.lrelu == 1) v = lrelu(v);
    if (o.r1) v = o.s1 * v + r1;
    if (o.lrelu == 3) v = r2 > 0.f ? v : 0.2f * v;
    else if (o.r2) v = o.s2 * v + r2;
    return v;
}

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

// Epilogue store phase shared by both kernels.  s_ep holds the tile's fp32 accumulators as [pixel q][channel] (pitch
// N + 4); r_first is the tall padded row of the tile's first output row.  Each thread owns one 8-channel group (so its
// bias is loaded once) and a fixed list of ITERS pixels; the loop is fully unrolled so every residual / LDS load of the
// tile is in flight before the first value is finished (the store phase is load-latency-bound otherwise), and the
// pixel -> (image, row) mapping walks the tall image without per-pixel divisions.  Planar fp32 output (HR_conv1 ->
// CEM): consecutive lanes take consecutive pixels of one channel plane.  Returns false if a split output left the
// f16 range.
__device__ __forceinline__ float split_at(const float *buf, long long pix, int cp, int ch) {
    const _Float16 *g = reinterpret_cast<const _Float16 *>(buf + pix * cp + (ch & ~7));
    return (float)g[ch & 7] + (float)g[8 + (ch & 7)];
}

// Output location of tile pixel q (tile rows of width tw from tall padded row r_first + 1, column x0): padded output
// pixel index, image, output row / column; false if q is past the tile, or on a halo row or past the batch.
__device__ __forceinline__ bool locate_q(const X3Params &p, int q, int r_first, int x0, int tw, int nq,
                                         long long &opix, int &b, int &oy, int &ox) {
    const esr_conv_out &o = p.o;
    const int HP = p.H + 2;
    const int b0 = r_first / HP;
    const int row = (tw == TWF) ? (q >> 5) : q / tw;
    const int col = q - row * tw;
    int yy = r_first + 1 + row - b0 * HP;
    b = b0;
    while (yy >= HP) {
        yy -= HP;
        ++b;
    }
    const int y = yy - 1;
    oy = o.out_sy * y + o.out_oy;
    ox = o.out_sx * (x0 + col) + o.out_ox;
    opix = ((long long)b * (o.out_h + 2) + oy + 1) * (long long)(o.out_w + 2) + ox + 1;
    return q < nq && b < p.B && y >= 0 && y < p.H;
}

// store_px: NTH_ cooperating threads (thread index t) store NPX consecutive pixels q0 .. q0+NPX-1 of the tile, whose
// accumulators s_ep holds in rows 0 .. NPX-1 (a whole tile by the workgroup, or one 32-pixel M-tile by its wave).
template <int N, int NTH_, int NPX>
__device__ __forceinline__ bool store_px(const X3Params &p, const float *s_ep, int q0, int r_first, int x0, int tw,
                                         int nq, int t) {
    constexpr int EP_P = N + 4;
    constexpr int GROUPS = N / 8;
    constexpr int PPI = NTH_ / GROUPS;         // pixels per iteration
    constexpr int ITERS = NPX / PPI;
    const esr_conv_out &o = p.o;
    auto locate = [&](int q, long long &opix, int &b, int &oy, int &ox) {
        return locate_q(p, q, r_first, x0, tw, nq, opix, b, oy, ox);
    };
    if (o.out_planar) {
        for (int it = t; it < NPX * p.cout; it += NTH_) {
            const int c = it / NPX, qq = it - c * NPX;
            long long opix;
            int b, oy, ox;
            if (!locate(q0 + qq, opix, b, oy, ox)) continue;
            float v = s_ep[qq * EP_P + c] * p.w_scale_inv + p.bias[c];
            v = epi(o, v, o.r1 ? split_at(o.r1, opix, o.r1_cp, o.r1_coff + c) : 0.f, o.r2 ? split_at(o.r2, opix, o.r2_cp, o.r2_coff + c) : 0.f);
            o.out[(((long long)b * p.cout + c) * o.out_h + oy) * o.out_w + ox] = v;
        }
        return true;
    }
    const int g = t % GROUPS;
    const int c = 8 * g;
    if (c >= p.cout) return true;
    float bk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bk[j] = (c + j < p.cout) ? p.bias[c + j] : 0.f;
    long long opix[ITERS];
    bool val[ITERS];
#pragma unroll
    for (int k = 0; k < ITERS; ++k) {
        int b, oy, ox;
        val[k] = locate(q0 + t / GROUPS + k * PPI, opix[k], b, oy, ox);
    }
    float r1v[ITERS][8], r2v[ITERS][8];
    if (o.r1) {
#pragma unroll
        for (int k = 0; k < ITERS; ++k)
            if (val[k]) load_group(reinterpret_cast<const unsigned char *>(o.r1) + (opix[k] * o.r1_cp + o.r1_coff + c) * 4,
                                   r1v[k]);
    }
    if (o.r2) {
#pragma unroll
        for (int k = 0; k < ITERS; ++k)
            if (val[k]) load_group(reinterpret_cast<const unsigned char *>(o.r2) + (opix[k] * o.r2_cp + o.r2_coff + c) * 4,
                                   r2v[k]);
    }
    bool ok = true;
#pragma unroll
    for (int k = 0; k < ITERS; ++k) {
        if (!val[k]) continue;
        const int qq = t / GROUPS + k * PPI;
        float v[8];
        const f32x4 v0 = *reinterpret_cast<const f32x4 *>(s_ep + qq * EP_P + c);
        const f32x4 v1 = *reinterpret_cast<const f32x4 *>(s_ep + qq * EP_P + c + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = v0[j]; v[j + 4] = v1[j]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            v[j] = v[j] * p.w_scale_inv + bk[j];
            v[j] = epi(o, v[j], o.r1 ? r1v[k][j] : 0.f, o.r2 ? r2v[k][j] : 0.f);
        }
        ok &= store_group(reinterpret_cast<unsigned char *>(o.out) + (opix[k] * o.out_cp + o.out_coff + c) * 4, v);
        if (o.out2)
            store_group(reinterpret_cast<unsigned char *>(o.out2) + (opix[k] * o.out2_cp + o.out2_coff + c) * 4, v);
    }
    return ok;
}

template <int N>
__device__ __forceinline__ bool store_tile(const X3Params &p, const float *s_ep, int r_first, int x0, int tw, int nq,
                                           int tid) {
    return store_px<N, NTHR, TH * TWF>(p, s_ep, 0, r_first, x0, tw, nq, tid);
}

template <int VM>
__device__ __forceinline__ void wait_vm_lgkm0() {
    static_assert(VM >= 0 && VM < 64, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(VM) : "memory");
}

// Workgroups are dispatched round-robin over the 8 XCDs (blockIdx b runs on XCD b % 8), each with its own L2.  With
// tiles numbered row-major, horizontally adjacent tiles then sit in different L2s and every tile's halo rows are
// fetched from HBM again by the XCD that owns the neighbour.  xcd_tile renumbers so that XCD x gets one contiguous
// run of tiles (a band of whole tile rows): vertical and horizontal neighbours share an L2, and the workgroups
// co-resident on an XCD at any moment cover a compact band.  A bijection for any grid size.
constexpr int N_XCD = 8;
__device__ __forceinline__ int xcd_tile(int b, int nb) {
    const int x = b % N_XCD, l = b / N_XCD, q = nb / N_XCD, r = nb % N_XCD;
    return x < r ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
}

// LDS byte address of a pointer into the kernel's __shared__ array
__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// One 16-byte LDS read the compiler does not track: the caller waits for it with lgkm_wait
__device__ __forceinline__ f16x8 ds_read16(uint32_t a) {
    f16x8 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
    return r;
}

template <int OFF>
__device__ __forceinline__ f16x8 ds_read16o(uint32_t a, int tap) {
    f16x8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
    (void)tap;
    return r;
}

// s_waitcnt lgkmcnt(N) that the K fragments pass through (the empty statements after it are ordered behind it), so
// no use of them is scheduled before the wait
template <int N, int K>
__device__ __forceinline__ void lgkm_wait(f16x8 (&f)[K]) {
    static_assert(N >= 0 && N < 16, "lgkmcnt");
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f[0]) : "i"(N));
#pragma unroll
    for (int i = 1; i < K; ++i) asm volatile("" : "+v"(f[i]));
}

// OS (one stage): a single LDS stage (input + weights, 57 KB at N = 32; the epilogue staging is the larger) and two
// workgroups per CU (4 waves per SIMD: <= 128 VGPRs; the second launch-bounds argument is waves per SIMD), so one
// workgroup's DMA waits, prologue and epilogue overlap the other's MFMAs.  THT: tile height (16: two 32-pixel M-tiles
// per wave; 8: one, which halves the accumulators and the epilogue staging so N = 64 also fits two per CU).
// DE (direct epilogue, N = 32): the MFMA operands are swapped (weights as A, pixels as B), so each lane ends with
// channels of ONE pixel; one v_permlane32_swap per register pair gathers 8 consecutive channels (one split group) per
// lane, and every lane finishes and stores its groups straight from registers: no LDS restage, no barrier.
template <int NT, int TS, bool ASMRD = true, int PFD = (NT == 1 ? 2 : 1), bool OS = false, int THT = TH,
          int WPS = (OS ? 4 : 1), bool DE = false, int DBGX = 0>
__global__ __launch_bounds__(NTHR, WPS) void conv_x3_kernel(X3Params p) {
    // DBGX (diagnostic builds, esr_x3_set_kernel 29 / 30; outputs are garbage): 1 = LDS-DMA of chunk 0 only, 2 = no
    // fragment reads / MFMAs
    static_assert(!DE || (NT == 1 && ASMRD), "direct epilogue: N = 32, explicit fragment reads");
    constexpr int MTW = THT / 8;  // M-tiles per wave
    constexpr int HYT = THT + 2;
    constexpr int IN_RECS_T = (HYT * HXF + 15) / 16 * 16;
    constexpr int T = TS * TS;
    constexpr int N = NT * 32;
    constexpr int W_RECS = T * N;
    constexpr int IN_B = IN_RECS_T * REC;
    constexpr int W_B = W_RECS * REC;
    constexpr int EP_P = N + 4;
    constexpr int EP_BYTES = THT * TWF * EP_P * 4;
    constexpr int NST = OS ? 1 : 2;  // LDS stages
    constexpr int LDS_BYTES = NST * (IN_B + W_B) > EP_BYTES ? NST * (IN_B + W_B) : EP_BYTES;
    static_assert(!OS || (WPS / 2) * LDS_BYTES <= 163840, "WPS / 2 workgroups per CU");
    constexpr int KIN = (IN_RECS_T / 16 + NWAVES - 1) / NWAVES;
    constexpr int KW = (W_RECS / 16 + NWAVES - 1) / NWAVES;
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int hl = lane >> 5;
    const int ml = lane & 31;

    const int tile = p.xcd_map ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tx = tile % p.tiles_x;
    const int ty = tile / p.tiles_x;
    const int x0 = tx * TWF;
    const int tw = min(TWF, p.W - x0);
    const int hx = tw + 2;
    const int r0 = ty * THT;
    const int rows_tot = p.B * (p.H + 2);
    const int nq = THT * tw;
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
        if (k < IN_RECS_T / 16 && r < HYT * hx && gy < rows_tot && gx < p.W + 2) {
            in_src[i] = (gy * rowp + gx) * pixb + (s << 4);
            in_hi[i] = s >> 1;
        }
    }
    // LDS-DMA piece q (0 .. KIN + KW - 1: input pieces, then weight pieces) of chunk j into stage st; pieces past the
    // tile are skipped (wave-uniform)
    auto dma_piece = [&](int j, int st, int q) {
        if (q < KIN) {
            const int k = wave + NWAVES * q;
            if (k >= IN_RECS_T / 16) return;
            const int groups = min(16, p.cin - 16 * j) >> 3;
            const void *src = (in_hi[q] >= 0 && in_hi[q] < groups) ? (const void *)(p.in + in_src[q] + 64LL * j)
                                                                   : (const void *)g_zero_page;
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(lds + st * IN_B + k * 1024), 16, 0, 0);
        } else {
            const int k = wave + NWAVES * (q - KIN);
            if (k >= W_RECS / 16) return;
            const int r = 16 * k + sub;
            const int s = ps ^ ((r >> 2) & 3);
            __builtin_amdgcn_global_load_lds((glob_void *)(p.w + (long long)j * W_B + r * REC + (s << 4)),
                                             (lds_void *)(lds + NST * IN_B + st * W_B + k * 1024), 16, 0, 0);
        }
    };
    auto dma = [&](int j, int st) {
#pragma unroll
        for (int q = 0; q < KIN + KW; ++q) dma_piece(j, st, q);
    };

    int aoff[T][MTW][2];
    bool mvalid[MTW];
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
        const int jm = MTW * wave + mt;
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

    f32x16 acc[MTW][NT];
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

    // Fragments are read X3_PF taps ahead of their MFMAs (X3_PF + 1 register sets): with one tap of lookahead the
    // reads of 8 waves (6-8 ds_read_b128 each) were covered by only ~5 of the wave's own MFMAs, and LDS latency
    // added to the matrix time instead of hiding under it.
    // Explicit ds_read_b128 fragment reads PFD taps ahead with counted lgkmcnt waits (see the ring kernel's
    // compute_asm); MFMAs unpredicated, the order per accumulator unchanged.  PFD = 2 needs 2 x NR < 16 (4-bit
    // lgkmcnt): N = 32 only.
    auto compute_asm = [&](const unsigned char *s_in, const unsigned char *s_w, auto &&hook) {
        constexpr int NR = 2 * MTW + 2 * NT;  // [ah0, al0, (ah1, al1), bh0, bl0, (bh1, bl1)]
        constexpr int NBUF = PFD + 1;
        static_assert(PFD * NR < 16, "lgkmcnt is a 4-bit count");
        // opaque stage bases: otherwise the per-stage fragment addresses are hoisted out of the chunk loop as 2 x 36
        // loop-invariant VGPRs (the N = 64 kernel then spills)
        uint32_t bi = lds_addr(s_in), bw = lds_addr(s_w);
        asm volatile("" : "+s"(bi), "+s"(bw));
        f16x8 f[NBUF][NR];
        auto ld = [&](int tap, int buf) {
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt) {
                // the lo slot is the hi slot ^ 1 (slot_off), i.e. byte offset ^ 16; stage bases are 1-KB aligned
                const uint32_t a = bi + aoff[tap][mt][0];
                f[buf][2 * mt] = ds_read16(a);
                f[buf][2 * mt + 1] = ds_read16(a ^ 16u);
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                f[buf][2 * MTW + 2 * nt] = ds_read16(bw + boff0 + (tap * N + nt * 32) * REC);
                f[buf][2 * MTW + 1 + 2 * nt] = ds_read16(bw + boff1 + (tap * N + nt * 32) * REC);
            }
        };
#pragma unroll
        for (int k = 0; k < PFD; ++k) ld(k, k);
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int cb = tap % NBUF;
            if (tap + PFD < T) ld(tap + PFD, (tap + PFD) % NBUF);
            const int ahead = min(PFD, T - 1 - tap);  // read groups still allowed in flight
            if (ahead >= 2) lgkm_wait<(PFD >= 2 ? 2 * NR : NR)>(f[cb]);
            else if (ahead == 1) lgkm_wait<NR>(f[cb]);
            else lgkm_wait<0>(f[cb]);
            f16x8 *q = f[cb];
            // (a, b) -> MFMA operands in the kernel's orientation: pixels x channels, or channels x pixels (DE)
            auto mma = [&](const f16x8 &a, const f16x8 &b, f32x16 &c) {
                if constexpr (DE) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c, 0, 0, 0);
                else c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
            };
            if constexpr ((DBGX & 8) != 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) mma(q[2 * mt + 1], q[2 * MTW + 2 * nt], acc[mt][nt]);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) mma(q[2 * mt], q[2 * MTW + 1 + 2 * nt], acc[mt][nt]);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) mma(q[2 * mt], q[2 * MTW + 2 * nt], acc[mt][nt]);
            if constexpr ((DBGX & 8) != 0) __builtin_amdgcn_s_setprio(0);
            hook(tap);  // e.g. the next chunk's LDS-DMA pieces, issued behind this tap's MFMAs
        }
    };
    auto compute = [&](const unsigned char *s_in, const unsigned char *s_w, auto &&hook) {
        if constexpr (ASMRD) {
            compute_asm(s_in, s_w, hook);
            return;
        }
        constexpr int NBUF = X3_PF + 1;
        f16x8 ah[NBUF][MTW], al[NBUF][MTW], bh[NBUF][NT], bl[NBUF][NT];
        auto ld = [&](int tap, int buf) {
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt) {
                ah[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + aoff[tap][mt][0]);
                al[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + aoff[tap][mt][1]);
            }
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                bh[buf][nt] = *reinterpret_cast<const f16x8 *>(s_w + (tap * N + nt * 32) * REC + boff0);
                bl[buf][nt] = *reinterpret_cast<const f16x8 *>(s_w + (tap * N + nt * 32) * REC + boff1);
            }
        };
#pragma unroll
        for (int k = 0; k < X3_PF; ++k)
            if (k < T) ld(k, k);
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int cb = tap % NBUF;
            if (tap + X3_PF < T) ld(tap + X3_PF, (tap + X3_PF) % NBUF);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[cb][mt], bh[cb][nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bl[cb][nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    if (mvalid[mt]) acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bh[cb][nt], acc[mt][nt], 0, 0, 0);
            hook(tap);
        }
    };

    // the explicit vmcnt(0) before each barrier: compute_asm's reads are invisible to the compiler's LDS-DMA tracking
    auto none = [](int) {};
    if constexpr (OS) {
        for (int j = 0; j < nchunk; ++j) {
            if (j) __syncthreads();  // every wave is done reading the stage
            if (!(DBGX & 1) || j == 0) dma(j, 0);
            wait_vm_lgkm0<0>();
            __syncthreads();
            if (mvalid[0] && !(DBGX & 2)) compute(lds, lds + IN_B, none);
        }
    } else {
    // IL (DBGX & 4): the next chunk's LDS-DMA pieces are spread over the first taps of this chunk, two behind each
    // tap's MFMAs, instead of issued as one burst before them (an LDS-DMA issue stalls the issuing wave ~60-180
    // cycles; as a burst both waves of a SIMD stall together and the matrix pipe idles)
    constexpr int NPC = KIN + KW;
    auto next = [&](int j, int st) {
        return [&, j, st](int tap) {
            if constexpr ((DBGX & 4) != 0) {
                if (j < nchunk && !(DBGX & 1)) {
                    constexpr int PER = (NPC + 4) / 5;  // pieces per tap over the first five taps
#pragma unroll
                    for (int e = 0; e < PER; ++e)
                        if (PER * tap + e < NPC) dma_piece(j, st, PER * tap + e);
                }
            }
        };
    };
    dma(0, 0);
    for (int j = 0; j < nchunk; j += 2) {
        wait_vm_lgkm0<0>();
        __syncthreads();
        if (!(DBGX & 4) && !(DBGX & 1) && j + 1 < nchunk) dma(j + 1, 1);
        if (mvalid[0] && !(DBGX & 2)) compute(lds, lds + 2 * IN_B, next(j + 1, 1));
        else if (DBGX & 4) for (int q = 0; q < NPC; ++q) if (j + 1 < nchunk && !(DBGX & 1)) dma_piece(j + 1, 1, q);
        if (j + 1 >= nchunk) break;
        wait_vm_lgkm0<0>();
        __syncthreads();
        if (!(DBGX & 4) && !(DBGX & 1) && j + 2 < nchunk) dma(j + 2, 0);
        if (mvalid[0] && !(DBGX & 2)) compute(lds + IN_B, lds + 2 * IN_B + W_B, next(j + 2, 0));
        else if (DBGX & 4) for (int q = 0; q < NPC; ++q) if (j + 2 < nchunk && !(DBGX & 1)) dma_piece(j + 2, 0, q);
    }
    }

    if constexpr (DE) {
        // acc[mt][0][r] = channel 8 (r >> 2) + 4 hl + (r & 3) of pixel 32 jm + ml.  Swapping registers r = 4..7 of
        // lanes 0-31 with r = 0..3 of lanes 32-63 (and r = 12..15 with 8..11) leaves every lane with channels
        // 8 (2 s + hl) + j in registers 8 s + j, j = 0..7: split groups 2 s + hl, s = 0, 1.
        const esr_conv_out &o = p.o;
        bool ok = true;
#pragma unroll
        for (int mt = 0; mt < MTW; ++mt) {
            if (!mvalid[mt]) continue;
            f32x16 &a = acc[mt][0];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    // v_permlane32_swap: lanes 32-63 of the first operand <-> lanes 0-31 of the second
                    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[8 * s + k]),
                                                                    __float_as_uint(a[8 * s + 4 + k]), false, false);
                    a[8 * s + k] = __uint_as_float(r[0]);
                    a[8 * s + 4 + k] = __uint_as_float(r[1]);
                }
            long long opix;
            int b, oy, ox;
            if (!locate_q(p, 32 * (MTW * wave + mt) + ml, r0, x0, tw, nq, opix, b, oy, ox)) continue;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int c = 8 * (2 * s + hl);
                if (c >= p.cout) continue;
                float v[8], r1v[8], r2v[8];
                if (!o.out_planar) {
                    if (o.r1) load_group(reinterpret_cast<const unsigned char *>(o.r1) + (opix * o.r1_cp + o.r1_coff + c) * 4, r1v);
                    if (o.r2) load_group(reinterpret_cast<const unsigned char *>(o.r2) + (opix * o.r2_cp + o.r2_coff + c) * 4, r2v);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        r1v[j] = (o.r1 && c + j < p.cout) ? split_at(o.r1, opix, o.r1_cp, o.r1_coff + c + j) : 0.f;
                        r2v[j] = (o.r2 && c + j < p.cout) ? split_at(o.r2, opix, o.r2_cp, o.r2_coff + c + j) : 0.f;
                    }
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    v[j] = a[8 * s + j] * p.w_scale_inv + ((c + j < p.cout) ? p.bias[c + j] : 0.f);
                    v[j] = epi(o, v[j], o.r1 ? r1v[j] : 0.f, o.r2 ? r2v[j] : 0.f);
                }
                if (o.out_planar) {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (c + j < p.cout) o.out[(((long long)b * p.cout + c + j) * o.out_h + oy) * o.out_w + ox] = v[j];
                } else {
                    ok &= store_group(reinterpret_cast<unsigned char *>(o.out) + (opix * o.out_cp + o.out_coff + c) * 4, v);
                    if (o.out2)
                        store_group(reinterpret_cast<unsigned char *>(o.out2) + (opix * o.out2_cp + o.out2_coff + c) * 4, v);
                }
            }
        }
        if (!ok && p.overflow) atomicOr(p.overflow, 1);
        return;
    }

    // ---- epilogue: restage fp32 accumulators as [pixel][channel] ----
    __syncthreads();
    float *s_ep = reinterpret_cast<float *>(lds);
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt) {
        if (!mvalid[mt]) continue;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int q = 32 * (MTW * wave + mt) + (r & 3) + 8 * (r >> 2) + 4 * hl;
                if (q < nq) s_ep[q * EP_P + nt * 32 + ml] = acc[mt][nt][r];
            }
    }
    __syncthreads();

    if constexpr ((DBGX & 16) != 0) return;  // diagnostic: no epilogue stores
    const bool ok = store_px<N, NTHR, THT * TWF>(p, s_ep, 0, r0, x0, tw, nq, tid);
    if (!ok && p.overflow) atomicOr(p.overflow, 1);
}

// ---- ring variant (N = 32, 3×3): two vertically adjacent tiles per workgroup, 3-deep input ring -------------------
//
// The classic kernel above re-stages each chunk's weights for every 512-pixel tile and waits for each chunk's DMA one
// compute phase after issuing it (two stages is all the LDS allows).  Here a workgroup owns tiles (tx, 2p) and
// (tx, 2p+1) and walks "units" u = (chunk u/2, tile u&1): the weights of a chunk are staged once for both tiles (half
// the weight bytes per FLOP), and LDS holds a 2-slot weight ring + a 3-slot input ring (2·18 KB + 3·39 KB = 153 KB), so
// every input tile and every weight chunk is fetched two units ahead.  The DMAs stay in flight across the barriers:
// each wave waits with a COUNTED vmcnt for exactly the data the next unit reads (all waves issue the same number of
// LDS-DMA instructions: short waves re-issue the last piece, rewriting identical bytes), then a raw s_barrier.
// Per accumulator the MFMA sequence is the classic kernel's, so the two kernels agree bit for bit.
constexpr int IN_PIECES = IN_RECS / 16;  // 1-KB LDS-DMA wave-instructions per input stage (39)


__device__ __forceinline__ void raw_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// DBG bits (diagnostic builds, esr_x3_set_kernel >= 3; outputs are garbage): 1 = no LDS-DMA in the main loop,
// 2 = no compute, 4 = fragment reads but no MFMAs, 8 = no barriers, 16 = slot 0 always (immediate LDS offsets),
// 32 = MFMAs not predicated on mvalid, 64 = no epilogue stores (accumulators kept live), 128 = no epilogue at all;
// 256 (valid outputs) = the compiler-scheduled fragment reads instead of compute_asm's (the pre-asm kernel, for A/B),
// 512 = compute_asm with lane-constant A addresses (timing probe for the address VALU work).
template <int NIN, bool STAG, int DBG = 0>
__global__ __launch_bounds__(NTHR, 1) void conv_x3_ring_kernel(X3Params p) {
    constexpr int T = 9;
    constexpr int N = 32;
    constexpr int W_RECS = T * N;
    constexpr int IN_B = IN_RECS * REC;
    constexpr int W_B = W_RECS * REC;
    constexpr int W_PIECES = W_RECS / 16;
    constexpr int EP_P = N + 4;
    constexpr int EP_BYTES = TH * TWF * EP_P * 4;
    constexpr int RING_BYTES = 2 * W_B + NIN * IN_B;
    constexpr int LDS_BYTES = RING_BYTES > EP_BYTES ? RING_BYTES : EP_BYTES;
    constexpr int KIN = (IN_PIECES + NWAVES - 1) / NWAVES;
    constexpr int KW = (W_PIECES + NWAVES - 1) / NWAVES;
    static_assert(LDS_BYTES <= 163840, "LDS");
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int hl = lane >> 5;
    const int ml = lane & 31;

    const int tx = blockIdx.x % p.tiles_x;
    const int tp = blockIdx.x / p.tiles_x;  // tile pair: tiles 2tp, 2tp+1
    const int x0 = tx * TWF;
    const int tw = min(TWF, p.W - x0);
    const int hx = tw + 2;
    const int r0 = 2 * tp * TH;
    const int rows_tot = p.B * (p.H + 2);
    const int nq = TH * tw;
    const int nmt = (nq + 31) >> 5;
    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;
    const long long tile_step = TH * rowp * pixb;
    const int nchunk = (p.cin + 15) >> 4;
    const int nunits = 2 * nchunk;

    const int sub = lane >> 2, ps = lane & 3;
    long long in_src[KIN];
    int in_hi[KIN], in_gy[KIN];
#pragma unroll
    for (int i = 0; i < KIN; ++i) {
        const int k = min(wave + NWAVES * i, IN_PIECES - 1);
        const int r = 16 * k + sub;
        const int s = ps ^ ((r >> 2) & 3);
        const int hy = r / hx, hxi = r - (r / hx) * hx;
        const int gy = r0 + hy, gx = x0 + hxi;
        in_hi[i] = -1;
        in_src[i] = 0;
        in_gy[i] = gy;
        if (r < HY * hx && gx < p.W + 2) {
            in_src[i] = (gy * rowp + gx) * pixb + (s << 4);
            in_hi[i] = s >> 1;
        }
    }
    auto dma_in = [&](int u, int slot) {
        const int j = u >> 1, t = u & 1;
        const int groups = min(16, p.cin - 16 * j) >> 3;
        unsigned char *dst = lds + 2 * W_B + slot * IN_B;
#pragma unroll
        for (int i = 0; i < KIN; ++i) {
            const int k = min(wave + NWAVES * i, IN_PIECES - 1);
            const bool ok = in_hi[i] >= 0 && in_hi[i] < groups && in_gy[i] + t * TH < rows_tot;
            const void *src =
                ok ? (const void *)(p.in + in_src[i] + t * tile_step + 64LL * j) : (const void *)g_zero_page;
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(dst + k * 1024), 16, 0, 0);
        }
    };
    auto dma_w = [&](int j, int slot) {
        const unsigned char *wj = p.w + (long long)j * W_B;
        unsigned char *dst = lds + slot * W_B;
#pragma unroll
        for (int i = 0; i < KW; ++i) {
            const int k = min(wave + NWAVES * i, W_PIECES - 1);
            const int r = 16 * k + sub;
            const int s = ps ^ ((r >> 2) & 3);
            __builtin_amdgcn_global_load_lds((glob_void *)(wj + r * REC + (s << 4)), (lds_void *)(dst + k * 1024), 16,
                                             0, 0);
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
            const int r = rec0 + (tap / 3) * hx + tap % 3;
            aoff[tap][mt][0] = slot_off(r, 2 * hl);
            aoff[tap][mt][1] = slot_off(r, 2 * hl + 1);
        }
    }
    const int bsw = (ml >> 2) & 3;
    const int boff0 = ml * REC + (((2 * hl) ^ bsw) << 4), boff1 = ml * REC + (((2 * hl + 1) ^ bsw) << 4);

    f32x16 acc[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[t][mt][r] = 0.f;

    // Fragment reads as explicit ds_read_b128 with COUNTED lgkmcnt waits: tap t+1's six reads are issued before tap
    // t's six MFMAs and the wait before those MFMAs leaves them in flight.  (The compiler's own schedule of the plain
    // loads sinks each read next to its MFMA and drains with lgkmcnt(0), which serialises LDS latency and the matrix
    // pipe.)  The MFMAs are not predicated on mvalid[1]: an invalid M-tile reads pixel 0's fragments and its
    // accumulator is never stored, and the wave with both M-tiles valid sets the barrier cadence anyway.
    auto compute_asm = [&](const unsigned char *s_in, const unsigned char *s_w, f32x16(&ac)[2]) {
        uint32_t bi = lds_addr(s_in), bw = lds_addr(s_w);
        asm volatile("" : "+s"(bi), "+s"(bw));  // keep the per-slot addresses from being hoisted (VGPRs)
        f16x8 f[2][6];  // [buf][ah0, al0, ah1, al1, bh, bl]
        uint32_t a0[2][2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            a0[mt][0] = bi + aoff[0][mt][0];
            a0[mt][1] = bi + aoff[0][mt][1];
        }
        auto ld = [&](int tap, int buf) {
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                if constexpr ((DBG & 512) != 0) {  // timing probe: lane-constant A addresses (wrong outputs)
                    f[buf][2 * mt] = ds_read16o<0>(a0[mt][0], tap);
                    f[buf][2 * mt + 1] = ds_read16o<0>(a0[mt][1], tap);
                } else {
                    f[buf][2 * mt] = ds_read16(bi + aoff[tap][mt][0]);
                    f[buf][2 * mt + 1] = ds_read16(bi + aoff[tap][mt][1]);
                }
            }
            f[buf][4] = ds_read16(bw + boff0 + tap * N * REC);
            f[buf][5] = ds_read16(bw + boff1 + tap * N * REC);
        };
        ld(0, 0);
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int cb = tap & 1;
            if (tap + 1 < T) {
                ld(tap + 1, cb ^ 1);
                lgkm_wait<6>(f[cb]);
            } else {
                lgkm_wait<0>(f[cb]);
            }
            f16x8 *q = f[cb];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(q[2 * mt + 1], q[4], ac[mt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(q[2 * mt], q[5], ac[mt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(q[2 * mt], q[4], ac[mt], 0, 0, 0);
        }
    };
    auto compute = [&](const unsigned char *s_in, const unsigned char *s_w, f32x16(&ac)[2]) {
        if constexpr ((DBG & (4 | 32 | 256)) == 0) {
            compute_asm(s_in, s_w, ac);
            return;
        }
        f16x8 ah[2][2], al[2][2], bh[2], bl[2];
        auto ld = [&](int tap, int buf) {
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                ah[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + aoff[tap][mt][0]);
                al[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + aoff[tap][mt][1]);
            }
            bh[buf] = *reinterpret_cast<const f16x8 *>(s_w + tap * N * REC + boff0);
            bl[buf] = *reinterpret_cast<const f16x8 *>(s_w + tap * N * REC + boff1);
        };
        ld(0, 0);
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int cb = tap & 1;
            if (tap + 1 < T) ld(tap + 1, cb ^ 1);
            if (DBG & 4) {
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) asm volatile("" ::"v"(ah[cb][mt]), "v"(al[cb][mt]));
                asm volatile("" ::"v"(bh[cb]), "v"(bl[cb]));
                continue;
            }
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
                if ((DBG & 32) || mvalid[mt]) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[cb][mt], bh[cb], ac[mt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
                if ((DBG & 32) || mvalid[mt]) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bl[cb], ac[mt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
                if ((DBG & 32) || mvalid[mt]) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bh[cb], ac[mt], 0, 0, 0);
        }
    };

    // Unit u: barrier; issue the input of unit u+NIN-1 (into the slot unit u-1 freed) and, on a tile-0 unit, the
    // weights of the next chunk (into the slot the previous chunk freed); compute; then wait until everything but
    // this unit's own batch has landed (NIN = 3: the next unit's input was issued one unit earlier), or (NIN = 2) all
    // but the weight prefetch.
    auto unit = [&](int u, f32x16(&ac)[2]) {
        if (!(DBG & 8)) raw_barrier();
        const bool bi = u + NIN - 1 < nunits;
        const bool bw = !(u & 1) && (u >> 1) + 1 < nchunk;
        auto issue = [&]() {
            if (DBG & 1) return;
            if (bi) dma_in(u + NIN - 1, (u + NIN - 1) % NIN);
            if (bw) dma_w((u >> 1) + 1, ((u >> 1) + 1) & 1);
        };
        // STAG: the two waves sharing a SIMD (w, w+4) issue their DMAs at opposite ends of the unit, so each one's
        // LDS-DMA issue runs beside the other's MFMAs (the batch is still >= one unit ahead of its consumer)
        const bool late = STAG && __builtin_amdgcn_readfirstlane(wave) >= NWAVES / 2;
        if (!late) issue();
        if (!(DBG & 2) && (mvalid[0] || (DBG & 32)))
            compute(lds + 2 * W_B + ((DBG & 16) ? 0 : (u % NIN)) * IN_B, lds + ((DBG & 16) ? 0 : ((u >> 1) & 1)) * W_B, ac);
        if (late) issue();
        if (u + 1 < nunits) {
            if (NIN == 3) {
                if (bi && bw) wait_vm_lgkm0<KIN + KW>();
                else if (bi) wait_vm_lgkm0<KIN>();
                else if (bw) wait_vm_lgkm0<KW>();
                else wait_vm_lgkm0<0>();
            } else {
                if (bw) wait_vm_lgkm0<KW>();
                else wait_vm_lgkm0<0>();
            }
        }
    };

    dma_in(0, 0);
    dma_w(0, 0);
    if (NIN == 3) {
        dma_in(1, 1);
        wait_vm_lgkm0<KIN>();
    } else {
        wait_vm_lgkm0<0>();
    }
    for (int j = 0; j < nchunk; ++j) {
        unit(2 * j, acc[0]);
        unit(2 * j + 1, acc[1]);
    }

    if (DBG & 128) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) asm volatile("" ::"v"(acc[t][mt]));
        return;
    }
    // ---- epilogue: restage both tiles' fp32 accumulators as [pixel][channel] (2 x 72 KB), then store ----
    static_assert(2 * EP_BYTES <= LDS_BYTES, "epilogue staging");
    float *s_ep = reinterpret_cast<float *>(lds);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            if (!mvalid[mt]) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int q = 32 * (2 * wave + mt) + (r & 3) + 8 * (r >> 2) + 4 * hl;
                if (q < nq) s_ep[t * (EP_BYTES / 4) + q * EP_P + ml] = acc[t][mt][r];
            }
        }
    __syncthreads();
    if (DBG & 64) return;
    bool ok = store_tile<N>(p, s_ep, r0, x0, tw, nq, tid);
    ok &= store_tile<N>(p, s_ep + EP_BYTES / 4, r0 + TH, x0, tw, nq, tid);
    if (!ok && p.overflow) atomicOr(p.overflow, 1);
}

// ---- persistent ring kernel (N = 32, 3×3) ---------------------------------------------------------------------------
//
// The ring kernel above still pays, per workgroup, a cold prologue (its first tiles come from HBM with nothing to
// overlap) and an epilogue whose 16 KB per wave of stores issue at ~7 B/cycle/CU while the matrix pipe idles; with three
// rounds of workgroups per launch that was ~15-20 % of an RDB conv (ablation in DESIGN.md §5).  Here one workgroup per
// CU walks its tile pairs (blockIdx.x, +gridDim.x, ...) as ONE stream of units: the 3-slot input ring and the 2-slot
// weight ring prefetch across pair boundaries (the next pair's first two input tiles and first weight chunk are in
// flight while the current pair finishes), and a pair's epilogue runs per wave — each wave restages its own 32-pixel
// M-tiles in the input slot the pair's last unit released and issues their stores, which then drain behind the next
// pair's MFMAs.  Fragments are read PF taps ahead; DMA addresses are 32-bit offsets from the fetched pair's first row
// and the lo halves of the A/B fragments are at offset ^ 16, which pays for the deeper fragment ring in registers.
// Per accumulator the MFMA sequence is the classic kernel's: results are bitwise identical.
// Measured (tools/x3_ring_ab.py, config-2 shapes): within ±3 % of the non-persistent ring kernel (prefetch 2) and
// slower at 96² — the store issue of the epilogue, not the cold prologue, is what the ring kernel loses per pair — so
// it is not selected by default (esr_x3_set_kernel 16 / 17).
template <int PF>
__global__ __launch_bounds__(NTHR, 1) void conv_x3_pring_kernel(X3Params p) {
    constexpr int NIN = 3;
    constexpr int T = 9;
    constexpr int N = 32;
    constexpr int W_RECS = T * N;
    constexpr int IN_B = IN_RECS * REC;
    constexpr int W_B = W_RECS * REC;
    constexpr int W_PIECES = W_RECS / 16;
    constexpr int EP_P = N + 4;
    constexpr int EPW_FLOATS = 32 * EP_P;  // one wave's restage area: one M-tile of 32 pixels
    constexpr int LDS_BYTES = 2 * W_B + NIN * IN_B;
    constexpr int KIN = (IN_PIECES + NWAVES - 1) / NWAVES;
    constexpr int KW = (W_PIECES + NWAVES - 1) / NWAVES;
    static_assert(NWAVES * EPW_FLOATS * 4 <= IN_B, "per-wave epilogue areas fit in one input slot");
    static_assert(LDS_BYTES <= 163840, "LDS");
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int hl = lane >> 5;
    const int ml = lane & 31;
    const int sub = lane >> 2, ps = lane & 3;
    const int npairs = p.tiles_x * ((p.tiles_y + 1) / 2);
    const int my_pairs = (npairs - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    if (my_pairs <= 0) return;
    const int nchunk = (p.cin + 15) >> 4;
    const int upp = 2 * nchunk;  // units per pair
    const int nunits = my_pairs * upp;
    const int rows_tot = p.B * (p.H + 2);
    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;
    const long long tile_step = TH * rowp * pixb;

    auto pair_geo = [&](int i, int &x0, int &tw, int &r0) {
        const int pr = (int)blockIdx.x + i * (int)gridDim.x;
        x0 = (pr % p.tiles_x) * TWF;
        tw = min(TWF, p.W - x0);
        r0 = 2 * (pr / p.tiles_x) * TH;
    };

    // LDS-DMA addressing of the pair being fetched (switches to the next pair ahead of the compute pair)
    int in_off[KIN], in_code[KIN];  // code = (halo row << 2) | (split group of the slot + 1); 0 = zero page
    int dma_pair = -1, dma_r0 = 0;
    auto set_dma = [&](int i) {
        int x0, tw, r0;
        pair_geo(i, x0, tw, r0);
        const int hx = tw + 2;
#pragma unroll
        for (int k = 0; k < KIN; ++k) {
            const int pc = min(wave + NWAVES * k, IN_PIECES - 1);
            const int r = 16 * pc + sub;
            const int s = ps ^ ((r >> 2) & 3);
            const int hy = r / hx;
            const int gx = x0 + r - hy * hx;
            const bool v = r < HY * hx && gx < p.W + 2;
            in_off[k] = v ? (int)((hy * rowp + gx) * pixb + (s << 4)) : 0;
            in_code[k] = v ? ((hy << 2) | ((s >> 1) + 1)) : 0;
        }
        dma_pair = i;
        dma_r0 = r0;
    };
    auto dma_in = [&](int v, int slot) {  // input of global unit v
        const int i = v / upp;
        if (i != dma_pair) set_dma(i);
        const int lv = v - i * upp;
        const int j = lv >> 1, t = lv & 1;
        const int groups = min(16, p.cin - 16 * j) >> 3;
        const unsigned char *base = p.in + (long long)dma_r0 * rowp * pixb + t * tile_step + 64LL * j;
        unsigned char *dst = lds + 2 * W_B + slot * IN_B;
#pragma unroll
        for (int k = 0; k < KIN; ++k) {
            const int pc = min(wave + NWAVES * k, IN_PIECES - 1);
            const int code = in_code[k];
            const bool ok = code != 0 && (code & 3) - 1 < groups && dma_r0 + (code >> 2) + t * TH < rows_tot;
            const void *src = ok ? (const void *)(base + in_off[k]) : (const void *)g_zero_page;
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(dst + pc * 1024), 16, 0, 0);
        }
    };
    auto dma_w = [&](int c, int slot) {  // weights of global chunk c (= chunk c % nchunk of every pair)
        const unsigned char *wj = p.w + (long long)(c % nchunk) * W_B;
        unsigned char *dst = lds + slot * W_B;
#pragma unroll
        for (int i = 0; i < KW; ++i) {
            const int k = min(wave + NWAVES * i, W_PIECES - 1);
            const int r = 16 * k + sub;
            const int s = ps ^ ((r >> 2) & 3);
            __builtin_amdgcn_global_load_lds((glob_void *)(wj + r * REC + (s << 4)), (lds_void *)(dst + k * 1024), 16,
                                             0, 0);
        }
    };

    // geometry of the pair being computed; fragment offsets of the hi halves (lo = offset ^ 16)
    int aoff[T][2];
    bool mvalid[2];
    int cx0 = 0, ctw = TWF, cr0 = 0, cnq = TH * TWF;
    auto set_geo = [&](int i) {
        pair_geo(i, cx0, ctw, cr0);
        const int hx = ctw + 2;
        cnq = TH * ctw;
        const int nmt = (cnq + 31) >> 5;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const int jm = 2 * wave + mt;
            mvalid[mt] = jm < nmt;
            int q = 32 * jm + ml;
            if (q >= cnq) q = 0;
            const int rec0 = (q / ctw) * hx + q % ctw;
#pragma unroll
            for (int tap = 0; tap < T; ++tap) aoff[tap][mt] = slot_off(rec0 + (tap / 3) * hx + tap % 3, 2 * hl);
        }
    };
    const int boff = ml * REC + (((2 * hl) ^ ((ml >> 2) & 3)) << 4);

    f32x16 acc[2][2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[t][mt][r] = 0.f;
    };

    auto compute = [&](const unsigned char *s_in, const unsigned char *s_w, f32x16(&ac)[2]) {
        constexpr int NBUF = PF + 1;
        f16x8 ah[NBUF][2], al[NBUF][2], bh[NBUF], bl[NBUF];
        auto ld = [&](int tap, int buf) {
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                ah[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + aoff[tap][mt]);
                al[buf][mt] = *reinterpret_cast<const f16x8 *>(s_in + (aoff[tap][mt] ^ 16));
            }
            bh[buf] = *reinterpret_cast<const f16x8 *>(s_w + tap * N * REC + boff);
            bl[buf] = *reinterpret_cast<const f16x8 *>(s_w + tap * N * REC + (boff ^ 16));
        };
#pragma unroll
        for (int k = 0; k < PF; ++k) ld(k, k);
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int cb = tap % NBUF;
            if (tap + PF < T) ld(tap + PF, (tap + PF) % NBUF);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
                if (mvalid[mt]) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[cb][mt], bh[cb], ac[mt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
                if (mvalid[mt]) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bl[cb], ac[mt], 0, 0, 0);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
                if (mvalid[mt]) ac[mt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[cb][mt], bh[cb], ac[mt], 0, 0, 0);
        }
    };

    auto unit = [&](int u, f32x16(&ac)[2]) {
        raw_barrier();
        const bool bi = u + NIN - 1 < nunits;
        if (bi) dma_in(u + NIN - 1, (u + NIN - 1) % NIN);
        const bool bw = !(u & 1) && (u >> 1) + 1 < (nunits >> 1);
        if (bw) dma_w((u >> 1) + 1, ((u >> 1) + 1) & 1);
        if (mvalid[0]) compute(lds + 2 * W_B + (u % NIN) * IN_B, lds + ((u >> 1) & 1) * W_B, ac);
        if (u + 1 < nunits) {
            if (bi && bw) wait_vm_lgkm0<KIN + KW>();
            else if (bi) wait_vm_lgkm0<KIN>();
            else if (bw) wait_vm_lgkm0<KW>();
            else wait_vm_lgkm0<0>();
        }
    };

    // per-wave epilogue of the pair just computed, staged in input slot `slot` (free: its unit has been consumed by
    // every wave, and its next DMA is issued only after the next unit's barrier)
    auto epilogue = [&](int slot) {
        float *s_ep = reinterpret_cast<float *>(lds + 2 * W_B + slot * IN_B) + wave * EPW_FLOATS;
        bool ok = true;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                if (!mvalid[mt]) continue;
#pragma unroll
                for (int r = 0; r < 16; ++r) s_ep[((r & 3) + 8 * (r >> 2) + 4 * hl) * EP_P + ml] = acc[t][mt][r];
                ok &= store_px<N, 64, 32>(p, s_ep, 32 * (2 * wave + mt), cr0 + t * TH, cx0, ctw, cnq, lane);
            }
        if (!ok && p.overflow) atomicOr(p.overflow, 1);
    };

    set_dma(0);
    dma_in(0, 0);
    dma_w(0, 0);
    dma_in(1, 1);
    wait_vm_lgkm0<KIN>();
    set_geo(0);
    zero_acc();
    for (int u = 0; u < nunits; u += 2) {
        unit(u, acc[0]);
        unit(u + 1, acc[1]);
        if ((u + 2) % upp == 0) {
            raw_barrier();
            epilogue((u + 1) % NIN);
            if (u + 2 < nunits) {
                set_geo((u + 2) / upp);
                zero_acc();
            }
        }
    }
}

// Narrow-N 3×3 conv (cout <= 3, planar fp32 output: HR_conv1 -> CEM, architecture.py:140-141).  An N = 32 MFMA tile
// would spend 29 of its 32 output columns on padding (10.7× the MFMA work), so the taps go into M instead: for every
// INPUT pixel p, Y[t·3 + o][p] = Σ_c W[o][c][t] · x[c][p] for the 9 taps t and 3 outputs o (27 of the 32 rows of one
// v_mfma_f32_32x32x16_f16 tile, K = 16 channels, N = 32 pixels of one padded row), then out[o][y][x] = Σ_t Y[t·3 + o]
// at the tap's neighbour — the tap shift moves from the K loop into a 9-term sum over an LDS image of Y.  Every input
// pixel is fetched once per tile straight into the B fragments (no LDS staging: each is used once), the 27×cin
// weights stay in registers as A fragments for the whole tile.  Tile = NR output rows × 30 columns of the tall padded
// batch image (input rows NR + 2 × 32 padded columns), 4 waves, input rows round-robin over the waves with the next
// row's fragments loaded under the current row's MFMAs.  HBM-bound: 4 B per input channel per pixel in, 12 B out.
constexpr int NR_ROWS = 16;             // output rows per tile
constexpr int NR_IN = NR_ROWS + 2;      // input rows per tile
constexpr int NR_COLS = 30;             // output columns per tile (input: 32 padded columns)
constexpr int NR_M = 27;                // 9 taps × 3 outputs
constexpr int NR_THR = 256;
constexpr int NR_LDS = NR_IN * NR_M * 32 * 4;  // Y image [row][m][32 columns] fp32: 62,208 B (two workgroups per CU)

template <int NCH>
__global__ __launch_bounds__(NR_THR, 2) void conv_x3_narrow_kernel(X3Params p) {
    __shared__ __attribute__((aligned(16))) float ys[NR_LDS / 4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hl = lane >> 5, ml = lane & 31;
    const int tile = p.xcd_map ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tx = tile % p.tiles_x, ty = tile / p.tiles_x;
    const int x0 = tx * NR_COLS;                  // first output column = first input padded column
    const int r0 = 1 + ty * NR_ROWS;              // first output tall padded row
    const int rows_tot = p.B * (p.H + 2);
    const long long rowp = (long long)(p.W + 2), pixb = 4LL * p.in_cp;

    // A fragments: row m = ml (tap m / 3, output m % 3), channels 8 hl .. +8 of chunk j (zero past cout / cin)
    f16x8 ah[NCH], al[NCH];
    {
        const int t = ml / 3, o = ml - 3 * (ml / 3);
        constexpr int N = 32, W_B = 9 * N * REC;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            ah[j] = f16x8{};
            al[j] = f16x8{};
            if (ml < NR_M && o < p.cout && 16 * j + 8 * hl < p.cin) {
                const unsigned char *w = p.w + (long long)j * W_B + (t * N + o) * REC + 32 * hl;
                ah[j] = *reinterpret_cast<const f16x8 *>(w);
                al[j] = *reinterpret_cast<const f16x8 *>(w + 16);
            }
        }
    }
    // B fragments of input row i (tall padded row r0 - 1 + i): pixel column x0 + ml, channels 16 j + 8 hl .. +8
    const int gx = x0 + ml;
    // Branch-free, so that the compiler counts the loads in flight (s_waitcnt vmcnt(N)) instead of draining them all at
    // the first MFMA: a lane past the image reads the clamped last row / column (its Y column is never summed into an
    // output), a channel group past cin reads group 0 of the same pixel (finite; its A rows are zero)
    const int gxc = min(gx, p.W + 1);
    auto load_row = [&](int i, f16x8 (&bh)[NCH], f16x8 (&bl)[NCH]) {
        const int gy = min(r0 - 1 + i, rows_tot - 1);
        const unsigned char *src = p.in + ((long long)gy * rowp + gxc) * pixb + 32 * hl;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            const unsigned char *s = src + (16 * j + 8 * hl < p.cin ? 64 * j : 0);
            bh[j] = *reinterpret_cast<const f16x8 *>(s);
            bl[j] = *reinterpret_cast<const f16x8 *>(s + 16);
        }
    };
    auto compute_row = [&](int i, const f16x8 (&bh)[NCH], const f16x8 (&bl)[NCH]) {
        f32x16 c = {};
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[j], bh[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[j], bl[j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[j], bh[j], c, 0, 0, 0);
        }
        // c[r] = Y[m = (r & 3) + 8 (r >> 2) + 4 hl][pixel ml]
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = (r & 3) + 8 * (r >> 2) + 4 * hl;
            if (m < NR_M) ys[(i * NR_M + m) * 32 + ml] = c[r];
        }
    };
    // rows wave, wave + 4, ... (wave-uniform bounds), PF of them in flight: with one row ahead a CU held ~32 KB of
    // loads in flight, about half what HBM's latency-bandwidth product asks for
    constexpr int RPW = (NR_IN + 3) / 4, PF = NCH <= 4 ? RPW : 3;
    // (loads unconditional — a wave's row past NR_IN reads a clamped row and is not computed — so that no branch
    // makes the waitcnt pass assume the worst)
    f16x8 bh[PF][NCH], bl[PF][NCH];
#pragma unroll
    for (int k = 0; k < PF; ++k) load_row(wave + 4 * k, bh[k], bl[k]);
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        if (wave + 4 * k < NR_IN) compute_row(wave + 4 * k, bh[k % PF], bl[k % PF]);
        if (k + PF < RPW) load_row(wave + 4 * (k + PF), bh[k % PF], bl[k % PF]);
    }
    __syncthreads();
    // out[o][y][x] = (Σ_{ky, kx} Y[3 (3 ky + kx) + o] at input row + ky, column + kx) / w_scale + bias
    const esr_conv_out &o = p.o;
    const int HP = p.H + 2;
    for (int idx = tid; idx < 3 * NR_ROWS * 32; idx += NR_THR) {
        const int col = idx & 31, row = (idx >> 5) % NR_ROWS, oc = idx / (32 * NR_ROWS);
        const int tr = r0 + row;
        if (oc >= p.cout || col >= NR_COLS || x0 + col >= p.W || tr >= rows_tot - 1) continue;
        const int b = tr / HP, y = tr - b * HP - 1;
        if (y < 0 || y >= p.H) continue;
        float s = 0.f;
#pragma unroll
        for (int t = 0; t < 9; ++t) s += ys[((row + t / 3) * NR_M + 3 * t + oc) * 32 + col + t % 3];
        const float v = s * p.w_scale_inv + p.bias[oc];
        const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * (x0 + col) + o.out_ox;
        o.out[(((long long)b * p.cout + oc) * o.out_h + oy) * o.out_w + ox] = v;
    }
}

int launch_x3(const void *in, int B, int H, int W, int in_cp, int cin, const void *w, const float *bias,
              float w_scale, int cout, int taps_side, int ty0, int tx0, const esr_conv_out *o, int *overflow,
              hipStream_t stream) {
    if (!in || !w || !bias || !o || !o->out) return ESR_EINVAL;
    if (B <= 0 || H <= 0 || W <= 0 || cin <= 0 || cout <= 0 || cout > 64 || !(w_scale > 0.f)) return ESR_EINVAL;
    if (cin % 8 || in_cp % 8 || in_cp < cin || !(o->lrelu == 0 || o->lrelu == 1 || (o->lrelu == 3 && o->r2)))
        return ESR_EINVAL;
    if (!o->out_planar && (cout % 8 || o->out_cp % 8 || o->out_coff % 8 || o->out_coff + cout > o->out_cp))
        return ESR_EINVAL;
    if ((o->r1 && (o->r1_cp % 8 || o->r1_coff % 8)) || (o->r2 && (o->r2_cp % 8 || o->r2_coff % 8)) ||
        (o->out2 && (o->out2_cp % 8 || o->out2_coff % 8)))
        return ESR_EINVAL;
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(w)) & 15) return ESR_EINVAL;
#ifdef ESR_X3_EXPERIMENTS
    // 85 / 86 (wider N = 32 3x3 tiles, below): every other conv as the automatic choice (variant 1)
    if ((g_x3_kernel >= 85 && g_x3_kernel <= 88) && !(taps_side == 3 && cout <= 32 && (!o->out_planar || g_x3_kernel == 88))) {
        const int saved = g_x3_kernel;
        g_x3_kernel = 1;
        const int rc = launch_x3(in, B, H, W, in_cp, cin, w, bias, w_scale, cout, taps_side, ty0, tx0, o, overflow,
                                 stream);
        g_x3_kernel = saved;
        return rc;
    }
#endif
    X3Params p;
    p.in = static_cast<const unsigned char *>(in);
    p.B = B; p.H = H; p.W = W; p.in_cp = in_cp; p.cin = cin;
    p.w = static_cast<const unsigned char *>(w);
    p.bias = bias; p.w_scale_inv = 1.f / w_scale; p.cout = cout;
    p.tap_y0 = ty0; p.tap_x0 = tx0;
    p.tiles_x = (W + TWF - 1) / TWF;
    p.tiles_y = (B * (H + 2) - 2 + TH - 1) / TH;
    p.xcd_map = g_tile_map;
    p.overflow = overflow;
    p.o = *o;
    const dim3 block(NTHR);
    if (g_x3_narrow && taps_side == 3 && cout <= 3 && o->out_planar && o->lrelu == 0 && !o->r1 && !o->r2 &&
        !o->out2 && cin <= 80 && (g_x3_kernel == 1 || g_x3_kernel == 63)) {
        X3Params q = p;
        q.tiles_x = (W + NR_COLS - 1) / NR_COLS;
        q.tiles_y = (B * (H + 2) - 2 + NR_ROWS - 1) / NR_ROWS;
        const dim3 gridn((unsigned)(q.tiles_x * q.tiles_y)), blockn(NR_THR);
        if (cin <= 64) hipLaunchKernelGGL((conv_x3_narrow_kernel<4>), gridn, blockn, 0, stream, q);
        else hipLaunchKernelGGL((conv_x3_narrow_kernel<5>), gridn, blockn, 0, stream, q);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    // Ring kernel (two tiles per workgroup, esr_x3_set_kernel 2): opt-in only.  With both kernels on counted-wait
    // fragment reads a ring pair cost ~2.0 two-stage classic tiles, and the one-stage classic kernel at two
    // workgroups per CU is faster still (tools/x3_ring_ab.py at config 2 / 3 shapes).
    const int tiles = p.tiles_x * p.tiles_y;
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0, v = 0;
        n_cu = (hipGetDevice(&dev) == hipSuccess &&
                hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
    }
    // N = 32 one-stage kernel, 16-row tiles at 2 workgroups per CU vs 8-row tiles at 3: a round of 8-row workgroups
    // takes ~3/4 of a round of 16-row ones (measured: at 148², where both grids fill their last round, 16-row is ~1 %
    // faster over a whole bench step; 8-row is 15-20 % faster at 96², where the 16-row grid's second round is nearly
    // empty), so compare rounds x 3 with rounds x 4, ties to 16-row
    const int tiles8 = p.tiles_x * ((B * (H + 2) - 2 + 7) / 8);
    const bool row8_pays = 3 * ((tiles8 + 3 * n_cu - 1) / (3 * n_cu)) < 4 * ((tiles + 2 * n_cu - 1) / (2 * n_cu));
#ifdef ESR_X3_EXPERIMENTS  // ring / persistent-ring variants: the ablation library only
    const int pairs = p.tiles_x * ((p.tiles_y + 1) / 2);
    if (taps_side == 3 && cout <= 32 && (g_x3_kernel == 16 || g_x3_kernel == 17)) {
        const dim3 gridp((unsigned)min(pairs, n_cu));
        if (g_x3_kernel == 16) hipLaunchKernelGGL((conv_x3_pring_kernel<1>), gridp, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3_pring_kernel<2>), gridp, block, 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if (taps_side == 3 && cout <= 32 && g_x3_kernel >= 2 && g_x3_kernel < 20) {
        const dim3 grid2((unsigned)pairs);
        switch (g_x3_kernel) {
        case 15: hipLaunchKernelGGL((conv_x3_ring_kernel<3, true>), grid2, block, 0, stream, p); break;
        case 18: hipLaunchKernelGGL((conv_x3_ring_kernel<3, false, 256>), grid2, block, 0, stream, p); break;
#ifdef ESR_X3_EXPERIMENTS  // ablations of the ring kernel (garbage outputs): the experiment library only
#define RING_DBG(v, bits) \
    case v: hipLaunchKernelGGL((conv_x3_ring_kernel<3, true, bits>), grid2, block, 0, stream, p); break;
        RING_DBG(3, 1)
        RING_DBG(4, 2)
        RING_DBG(5, 4)
        RING_DBG(6, 1 | 8)
        RING_DBG(7, 1 | 16)
        RING_DBG(8, 1 | 32)
        RING_DBG(9, 1 | 8 | 16 | 32)
        RING_DBG(10, 4 | 1)
        RING_DBG(11, 4 | 1 | 64)
        RING_DBG(12, 4 | 1 | 128)
        RING_DBG(13, 64)
        RING_DBG(14, 2 | 128)
        case 19: hipLaunchKernelGGL((conv_x3_ring_kernel<3, false, 512>), grid2, block, 0, stream, p); break;
#undef RING_DBG
#endif
        default: hipLaunchKernelGGL((conv_x3_ring_kernel<3, false>), grid2, block, 0, stream, p);
        }
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#endif
    const dim3 grid((unsigned)(p.tiles_x * p.tiles_y));
    // Default (variant 1) since round 2: the column-tile kernel (esr_conv_x3c.hip) for 3x3 convs with cout > 32, and
    // with cout <= 32 where the 16-row classic grid fills its rounds (2-6 % faster per launch at the config-2/3
    // shapes, bitwise identical; profiles/r2_x3c_ab.txt); where 8-row classic tiles at three workgroups per CU pay
    // (small grids), the classic kernel stays.  Variant 24 = the round-1 automatic choice (classic only).
    // the polyphase upconv phases (2x2 taps) too: 341 -> 287 us per config-2 launch (whole-step A/B, 2 rounds)
    // N = 32 12-column tiles (three workgroups per CU) also where the classic 8-row tiles look better by rounds, once
    // the 12-column grid has a tile per CU: config 3 (B=16 × 96², 392 tiles) 1.00-1.07× per launch, 135.7 -> 133.9-
    // 134.8 ms per step; config 5 (B=8 × 172², 660 tiles) 1.09-1.12×; HR_conv1 at 592² 1115 -> 1060 us.  Below a tile
    // per CU (B=8 × 64²: 102 tiles) the 8-row tiles stay (0.70-0.73× there; profiles/r4_x3_n32_grid_ab.txt)
    const int tiles12 = ((W + 11) / 12) * ((B * (H + 2) - 2 + 31) / 32);
    const bool x3c_pays = taps_side == 2 || (taps_side == 3 && (cout > 32 || !row8_pays || tiles12 >= n_cu));
    if ((g_x3_kernel >= 50 && g_x3_kernel <= 62) || g_x3_kernel == 64 || g_x3_kernel == 65 ||
        (g_x3_kernel >= 70 && g_x3_kernel <= 88) ||
        ((g_x3_kernel == 1 || g_x3_kernel == 63) && x3c_pays)) {
        X3cParams c;
        c.in = p.in; c.B = B; c.H = H; c.W = W; c.in_cp = in_cp; c.cin = cin; c.w = p.w; c.bias = bias;
        c.w_scale_inv = p.w_scale_inv; c.cout = cout; c.tap_y0 = ty0; c.tap_x0 = tx0; c.tiles_x = c.tiles_y = 0;
        c.xcd_map = g_tile_map; c.overflow = overflow; c.o = *o;
        c.w_ld = c.w_roff = 0;
        c.w_cstride = 0;
        // N = 64 3×3 convs: 12-column tiles (four 3-column waves, two workgroups per CU) where their rounds cost less
        // than the 16-column tiles' (12·⌈t12/2CU⌉ < 16·⌈t16/2CU⌉): 1.08× the N split at config 3's 96², 1.10× at
        // 154², 1.05–1.24× at smaller grids; 16-column tiles at 172² (one round vs two: 1.18× the split) and 148²
        // (a tie); profiles/r4_x3_n64_tiles.txt.  Round 3's N split (two N = 32 launches) lost to one of the two at
        // every measured grid and is the ablation library's option (esr_x3_set_nsplit)
#ifdef ESR_X3_EXPERIMENTS  // 70-74: the persistent double-buffered N = 32 kernel (esr_conv_x3p.hip) and its ablations
        if ((g_x3_kernel == 85 || g_x3_kernel == 86) && taps_side == 3 && cout <= 32 && !o->out_planar)
            return x3c_launch(c, taps_side, stream, g_x3_kernel == 85 ? 300 : 301);  // wider N = 32 tiles (A/B)
        if (g_x3_kernel == 87 && taps_side == 3 && cout <= 32 && !o->out_planar)
            return x3c_launch(c, taps_side, stream, 302);  // stamped diagnostic build of the 12-column kernel
        if (g_x3_kernel == 88 && taps_side == 3 && cout <= 32)
            return x3c_launch(c, taps_side, stream, 303);  // 8-channel double-buffered form (A/B)
        if (g_x3_kernel >= 80 && g_x3_kernel <= 84 && cout <= 32) {  // 12-column time split: 81 = no DMA after chunk 0
            // + no stores, 82 = 81 without MFMAs (reads only), 83 = 81 without reads (MFMAs only), 84 = neither
            static const int dbgt[5] = {64, 5, 13, 21, 29};  // 64: the kernel as built (DBG 0)
            return x3c_launch(c, taps_side, stream, 256 * dbgt[g_x3_kernel - 80]);
        }
        if (g_x3_kernel >= 70 && g_x3_kernel <= 79) {  // 75-79: two-column waves (64 x 8 tiles)
            static const int dbgp[5] = {0, 1, 2, 4, 5};
            const int v = g_x3_kernel - 70;
            if (taps_side == 3 && cout <= 32 && !o->out_planar)
                return x3p_launch(c, stream, dbgp[v % 5] | (v >= 5 ? 16 : 0));
            return x3c_launch(c, taps_side, stream, cout > 32 ? 0 : 128);
        }
#endif
        const int rows32 = (B * (H + 2) - 2 + 31) / 32;
        const int tiles16 = ((W + 15) / 16) * rows32;
        if (taps_side == 3 && cout > 32 && (g_x3_kernel == 1 || g_x3_kernel == 63) && !o->out_planar) {
            const int t12 = ((W + 11) / 12) * rows32;
            const int r12 = (t12 + 2 * n_cu - 1) / (2 * n_cu), r16 = (tiles16 + 2 * n_cu - 1) / (2 * n_cu);
            if (12 * r12 < 16 * r16) return x3c_launch(c, taps_side, stream, 129);
        }
        if (g_x3_nsplit && taps_side == 3 && cout > 32 && (g_x3_kernel == 1 || g_x3_kernel == 63) &&
            tiles16 < 2 * n_cu && !o->out_planar) {
            for (int h = 0; h < 2; ++h) {
                X3cParams ch = c;
                ch.cout = min(32, cout - 32 * h);
                ch.bias = bias + 32 * h;
                ch.w_ld = 64;                                    // the N = 64 packing: 64 records per tap
                ch.w_roff = 32 * h;
                ch.w_cstride = 9LL * 64 * 64;                    // 9 taps × 64 records × 64 B per 16-channel chunk
                ch.o.out_coff += 32 * h;
                if (ch.o.r1) ch.o.r1_coff += 32 * h;
                if (ch.o.r2) ch.o.r2_coff += 32 * h;
                if (ch.o.out2) ch.o.out2_coff += 32 * h;
                const int rc = x3c_launch(ch, taps_side, stream, 128);
                if (rc != ESR_OK) return rc;
            }
            return ESR_OK;
        }
#ifdef ESR_X3_EXPERIMENTS
        if (g_x3_kernel == 65) return x3c_launch(c, taps_side, stream, cout > 32 ? 129 : 128);  // N = 64 in 12 columns
        if (g_x3_kernel == 60) return x3c_launch(c, taps_side, stream, 16);
        if (g_x3_kernel == 61) return x3c_launch(c, taps_side, stream, 32);
        if (g_x3_kernel == 62) return x3c_launch(c, taps_side, stream, 64);
#endif
        // N = 32 3×3 convs (the RDB growth convs): 12-column tiles of four 3-column waves at three workgroups per CU
        // (variant 64; 0.9 % per config-2 step over the 16-column tiles of variant 50, bitwise equal)
        if (g_x3_kernel == 64 || ((g_x3_kernel == 1 || g_x3_kernel == 63) && taps_side == 3 && cout <= 32))
            return x3c_launch(c, taps_side, stream, 128);
#ifdef ESR_X3_EXPERIMENTS  // 51-54: x3c ablations, 55-59: the warp-specialised persistent form and its ablations
        static const int dbg[5] = {0, 1, 2, 4, 5};
        if (g_x3_kernel >= 55 && g_x3_kernel <= 59) return x3s_launch(c, taps_side, stream, dbg[g_x3_kernel - 55]);
        return x3c_launch(c, taps_side, stream, g_x3_kernel >= 50 && g_x3_kernel <= 54 ? dbg[g_x3_kernel - 50] : 0);
#else
        return x3c_launch(c, taps_side, stream, 0);
#endif
    }
#ifdef ESR_X3_EXPERIMENTS  // DBGX ablations of the classic kernel (40-46; 29/30 below), garbage outputs
    if (taps_side == 3 && g_x3_kernel >= 40 && g_x3_kernel < 50) {
#define XV(NT_, fl) hipLaunchKernelGGL((conv_x3_kernel<NT_, 3, true, (NT_ == 1 ? 2 : 1), false, TH, 1, false, fl>), grid, block, 0, stream, p)
        const bool n64 = cout > 32;
        switch (g_x3_kernel) {
        case 40: if (n64) XV(2, 4); else XV(1, 4); break;
        case 41: if (n64) XV(2, 4 | 8); else XV(1, 4 | 8); break;
        case 42: if (n64) XV(2, 1); else XV(1, 1); break;
        case 43: if (n64) XV(2, 2); else XV(1, 2); break;
        case 44: if (n64) XV(2, 16); else XV(1, 16); break;
        case 45: if (n64) XV(2, 8); else XV(1, 8); break;
        case 46: if (n64) XV(2, 4 | 16); else XV(1, 4 | 16); break;
        default: if (n64) XV(2, 0); else XV(1, 0);
        }
#undef XV
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if (taps_side == 3 && cout <= 32 && (g_x3_kernel == 29 || g_x3_kernel == 30)) {
        // the 16-row one-stage kernel: 29 = no LDS-DMA after chunk 0, 30 = no compute
        if (g_x3_kernel == 29) hipLaunchKernelGGL((conv_x3_kernel<1, 3, true, 1, true, TH, 4, false, 1>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3_kernel<1, 3, true, 1, true, TH, 4, false, 2>), grid, block, 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#endif
#ifdef ESR_X3_EXPERIMENTS  // bitwise-identical A/B variants of the classic kernel
    if (taps_side == 3 && g_x3_kernel == 20) {  // A/B: the classic kernel with compiler-scheduled fragment reads
        if (cout > 32) hipLaunchKernelGGL((conv_x3_kernel<2, 3, false>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3_kernel<1, 3, false>), grid, block, 0, stream, p);
    } else if (taps_side == 3 && cout <= 32 && g_x3_kernel == 21) {  // A/B: N = 32 with prefetch distance 1
        hipLaunchKernelGGL((conv_x3_kernel<1, 3, true, 1>), grid, block, 0, stream, p);
    } else if (taps_side == 3 && cout > 32 && g_x3_kernel == 23) {
        // A/B: N = 64 with 8-row tiles, one stage, two workgroups per CU (prefetch 2 would spill at 128 VGPRs)
        p.tiles_y = (B * (H + 2) - 2 + 7) / 8;
        const dim3 grid8((unsigned)(p.tiles_x * p.tiles_y));
        hipLaunchKernelGGL((conv_x3_kernel<2, 3, true, 1, true, 8>), grid8, block, 0, stream, p);
    } else if (taps_side == 3 && cout <= 32 && (g_x3_kernel == 27 || g_x3_kernel == 28)) {
        // N = 32 with the direct (register) epilogue: 27 = 16-row tiles at two workgroups per CU, 28 = 8-row at three
        if (g_x3_kernel == 28) {
            p.tiles_y = (B * (H + 2) - 2 + 7) / 8;
            const dim3 grid8((unsigned)(p.tiles_x * p.tiles_y));
            hipLaunchKernelGGL((conv_x3_kernel<1, 3, true, 1, true, 8, 6, true>), grid8, block, 0, stream, p);
        } else {
            hipLaunchKernelGGL((conv_x3_kernel<1, 3, true, 1, true, TH, 4, true>), grid, block, 0, stream, p);
        }
    } else if (taps_side == 3 && cout <= 32 && g_x3_kernel == 22) {  // A/B: two stages, one workgroup per CU (16 rows)
        hipLaunchKernelGGL((conv_x3_kernel<1, 3>), grid, block, 0, stream, p);
    } else
#endif
    if (taps_side == 3 && cout <= 32 && g_x3_kernel != 22 && g_x3_kernel != 26 && (g_x3_kernel == 25 || row8_pays)) {
        // N = 32 with 8-row tiles (one 32-pixel M-tile per wave), one stage, three workgroups per CU (<= 80 VGPRs)
        p.tiles_y = (B * (H + 2) - 2 + 7) / 8;
        const dim3 grid8((unsigned)(p.tiles_x * p.tiles_y));
        hipLaunchKernelGGL((conv_x3_kernel<1, 3, true, 1, true, 8, 6>), grid8, block, 0, stream, p);
    } else if (taps_side == 3) {
        // N = 32 with 16-row tiles (variant 26, or where row8_pays is false): one LDS stage and two workgroups per CU
        // (7-14 % faster than two stages and one workgroup at the config-2/3 shapes, profiles/r1_x3_reads_ab.txt);
        // N = 64 stays at one double-buffered 16-row workgroup per CU (variant 23, 8-row tiles at two per CU: 8 %
        // faster at 96², 4 % slower at 148²)
        if (cout > 32) hipLaunchKernelGGL((conv_x3_kernel<2, 3>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3_kernel<1, 3, true, 1, true>), grid, block, 0, stream, p);
    } else {
        if (cout > 32) hipLaunchKernelGGL((conv_x3_kernel<2, 2>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3_kernel<1, 2>), grid, block, 0, stream, p);
    }
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

}  // namespace

extern "C" int esr_conv3x3_fwd_x3(const void *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                                  const void *w_packed, const float *bias, float w_scale, int32_t cout,
                                  const esr_conv_out *o, int32_t *overflow, esr_stream_t stream) {
    return launch_x3(in, B, H, W, in_cp, cin, w_packed, bias, w_scale, cout, 3, 0, 0, o, overflow,
                     (hipStream_t)stream);
}

extern "C" int esr_upconv2x_phase_fwd_x3(const void *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                                         const void *w_packed, const float *bias, float w_scale, int32_t cout,
                                         int32_t py, int32_t px, const esr_conv_out *o, int32_t *overflow,
                                         esr_stream_t stream) {
    if (py < 0 || py > 1 || px < 0 || px > 1) return ESR_EINVAL;
    return launch_x3(in, B, H, W, in_cp, cin, w_packed, bias, w_scale, cout, 2, py, px, o, overflow,
                     (hipStream_t)stream);
}

extern "C" int esr_hr_convs_x3(const void *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t zc,
                               const void *w0, const float *bias0, float w0_scale, const void *w1, float *y,
                               int32_t *overflow, esr_stream_t stream) {
    if (!in || !w0 || !bias0 || !w1 || !y || B <= 0 || H <= 0 || W <= 0 || (zc != 0 && zc != 8) || in_cp != zc + 64 ||
        !(w0_scale > 0.f))
        return ESR_EINVAL;
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(w0) | reinterpret_cast<uintptr_t>(w1) |
         reinterpret_cast<uintptr_t>(y)) & 15)
        return ESR_EINVAL;
    X3cParams c = {};
    c.in = static_cast<const unsigned char *>(in);
    c.B = B; c.H = H; c.W = W; c.in_cp = in_cp; c.cin = in_cp;
    c.w = static_cast<const unsigned char *>(w0);
    c.bias = bias0; c.w_scale_inv = 1.f / w0_scale; c.cout = 64;
    c.xcd_map = g_tile_map; c.overflow = overflow;
    c.o.lrelu = 1;
    c.w1 = static_cast<const unsigned char *>(w1);
    c.y1 = y;
    c.zc1 = zc;
    return x3c_launch_hr1(c, (hipStream_t)stream);
}

extern "C" int esr_hr1_sum(const float *y, int32_t B, int32_t H, int32_t W, const float *bias1, float scale_inv,
                           float *out, esr_stream_t stream) {
    if (!y || !bias1 || !out || B <= 0 || H <= 0 || W <= 0 || (reinterpret_cast<uintptr_t>(y) & 15)) return ESR_EINVAL;
    return hr1_sum_launch(y, B, H, W, bias1, scale_inv, out, (hipStream_t)stream);
}
