// esr_conv_x3p.hip — x3 (split-f16) 3×3 convolution, N = 32: persistent, double-buffered column-tile form.
// ABLATION LIBRARY ONLY (round 5 experiment, profiles/r5_x3p_ab.txt: 0.95x the production kernel with the epilogue
// restaged through LDS, 0.6-0.8x with the deferred register epilogue below).
//
// Same numerics, layouts, fragment sweep and epilogue contract as the column-tile kernel (esr_conv_x3c.hip; read its
// header first) and bitwise equal to it: every accumulator receives the same MFMAs in the same order.  What differs
// is the dataflow around the sweep:
//
//  * Persistent: one 8-wave workgroup per CU walks a run of tiles (its XCD's contiguous band, x3p_tile), as one stream
//    of units u = (tile, 16-channel K chunk).  Unit u+1's input halo and weights are LDS-DMA'd into the other of two
//    LDS stages while unit u is computed, so the matrix cores do not wait for a chunk's loads, across tile boundaries
//    included (a tile's epilogue runs while the next tile's first chunk lands).  One barrier per unit.
//  * Bigger tiles: 64 rows × 12 columns (waves (h, g): row half h of 32 MFMA rows, column group g of 3 columns), so a
//    staged weight chunk feeds 768 output pixels instead of 384 and the halo is 66 × 14 instead of 34 × 14: 101 staged
//    bytes per output pixel and chunk (the 12-column one-stage kernel: 127).
//  * LDS: 2 × (59,392 B input + 18,432 B weights) = 155,648 B.
//  * Epilogue from registers (MFMA operands swapped so each lane holds one pixel's channels, one permlane32 swap per
//    register pair: esr_conv_x3.hip's direct epilogue), deferred by one unit: a tile's stores are issued during the
//    next tile's first chunk, by one wave of each SIMD before its MFMAs and by the other after them.
#include <hip/hip_runtime.h>
#include <type_traits>
#include "esr_amd.h"
#include "esr_x3c.h"

#ifdef ESR_X3_EXPERIMENTS  // measured slower than the production dispatch (profiles/r5_x3p_ab.txt): ablation library only

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glob_void;

constexpr int REC = 64;                           // bytes per staged record: 16 channels, split
constexpr int PT = 64;                            // tile rows (two 32-row M-tiles)
constexpr int NG = 4;                             // column groups
constexpr int NWV = 2 * NG;                       // waves (8)
constexpr int NTHR = 64 * NWV;
constexpr int HY = PT + 2;                        // 66 halo rows
constexpr int N = 32;
constexpr int T = 9;
constexpr int W_RECS = T * N;                     // 288
constexpr int W_PIECES = W_RECS / 16;             // 18
constexpr int KW = (W_PIECES + NWV - 1) / NWV;    // 3
constexpr int W_B = W_RECS * REC;                 // 18,432
constexpr int N_XCD = 8;

// CW output columns per wave: tiles of 64 rows × 4·CW columns (CW = 3: 12 columns, 66 × 14 halo)
template <int CW> struct X3pShape {
    static constexpr int PC = NG * CW;                           // tile columns
    static constexpr int HX = PC + 2;                            // halo columns
    static constexpr int IN_RECS = HY * HX;
    static constexpr int IN_PIECES = (IN_RECS + 15) / 16;        // one-KB LDS-DMA wave-instructions
    static constexpr int IN_B = IN_PIECES * 16 * REC;
    static constexpr int KIN = (IN_PIECES + NWV - 1) / NWV;      // input pieces per wave
    static constexpr int STAGE = IN_B + W_B;
    static constexpr int NIC = CW + 2;                           // halo columns a wave reads
    static constexpr int NSTEP = NIC * 3;                        // A steps (halo column, tap row) per sweep
    static_assert(2 * STAGE <= 163840, "two LDS stages");
};

__device__ __attribute__((aligned(16))) unsigned char g_zero64p[64];

__device__ __forceinline__ float lrelu(float v) { return v > 0.f ? v : 0.2f * v; }

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

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

template <int OFF>
__device__ __forceinline__ f16x8 ds_read16(uint32_t a) {
    static_assert(OFF >= 0 && OFF < 65536, "ds_read offset");
    f16x8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
    return r;
}

template <int NW>
__device__ __forceinline__ void lgkm_wait2(f16x8 &a, f16x8 &b) {
    static_assert(NW >= 0 && NW < 16, "lgkmcnt");
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(NW));
}

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

template <int I, int E, class F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, E>(f);
    }
}

// k-th tile of workgroup b in a grid of g: XCD x = b % 8 owns the contiguous band [x q, (x+1) q) of tiles
// (q = ceil(ntiles / 8)), dealt round-robin to its workgroups, so the tiles in flight on one XCD are neighbours and
// share halo lines in its L2; -1 past the end
__device__ __forceinline__ int x3p_tile(int b, int g, int ntiles, int k) {
    const int x = b % N_XCD, l = b / N_XCD;
    const int per = (g - x + N_XCD - 1) / N_XCD;
    const int q = (ntiles + N_XCD - 1) / N_XCD;
    const int t = l + k * per;
    return (t < q && x * q + t < ntiles) ? x * q + t : -1;
}

// DBG (ablation library only, garbage outputs): 1 = no LDS-DMA after the first unit, 2 = no fragment reads / MFMAs,
// 4 = no epilogue stores
template <int DBG = 0, int CW = 3>
__global__ __launch_bounds__(NTHR, 2) void conv_x3p_kernel(X3cParams p) {
    using S = X3pShape<CW>;
    constexpr int PC = S::PC, IN_RECS = S::IN_RECS, IN_PIECES = S::IN_PIECES, IN_B = S::IN_B, KIN = S::KIN;
    constexpr int STAGE = S::STAGE, NIC = S::NIC, NSTEP = S::NSTEP;
    __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wh = wave / NG;          // row half: MFMA rows 32·wh .. +31 of the tile
    const int wg = wave % NG;          // column group: tile columns CW·wg .. +CW-1
    const int hl = lane >> 5;
    const int ml = lane & 31;
    const int ntiles = p.tiles_x * p.tiles_y;
    const int rows_tot = p.B * (p.H + 2);
    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;
    const int nchunk = (p.cin + 15) >> 4;

    // ---- LDS-DMA addressing, tile-relative: input piece q of this wave = records 16 (wave + 8 i) .. +15 ----
    const int sub = lane >> 2, ps = lane & 3;
    unsigned in_off[KIN];  // byte offset from the tile origin (slot included, bit 1 = second 8-channel group)
#pragma unroll
    for (int i = 0; i < KIN; ++i) {
        const int q = wave + NWV * i;
        const int r = 16 * q + sub;
        const int hx = r / HY, hy = r - (r / HY) * HY;
        const int s = ps ^ ((hy >> 2) & 3);
        in_off[i] = (unsigned)((hy * rowp + hx) * pixb + (s << 4)) | ((s >> 1) << 1);
    }
    // per tile: bit i set = this lane's record of piece i lies inside the tall image (rows) and the padded width
    auto in_mask = [&](int tile) {
        const int x0 = (tile % p.tiles_x) * PC, r0 = (tile / p.tiles_x) * PT;
        unsigned m = 0;
#pragma unroll
        for (int i = 0; i < KIN; ++i) {
            const int q = wave + NWV * i;
            const int r = 16 * q + sub;
            const int hx = r / HY, hy = r - (r / HY) * HY;
            if (q < IN_PIECES && r < IN_RECS && r0 + hy < rows_tot && x0 + hx < p.W + 2) m |= 1u << i;
        }
        return m;
    };
    const long long w_cs = p.w_cstride ? p.w_cstride : (long long)W_B;
    const int w_ld = p.w_ld ? p.w_ld : N;
    auto dma = [&](int tile, unsigned mask, int j, int stage) {
        const int x0 = (tile % p.tiles_x) * PC, r0 = (tile / p.tiles_x) * PT;
        const unsigned char *tile_in = p.in + ((long long)r0 * rowp + x0) * pixb + 64LL * j;
        const int groups = min(16, p.cin - 16 * j) >> 3;  // 8-channel groups present in the chunk (1 or 2)
        unsigned char *st = lds + stage * STAGE;
#pragma unroll
        for (int i = 0; i < KIN; ++i) {
            const int q = wave + NWV * i;
            if (q >= IN_PIECES) break;
            const unsigned o = in_off[i];
            const bool ok = ((mask >> i) & 1u) && ((o >> 1) & 1u) < (unsigned)groups;
            const void *src = ok ? (const void *)(tile_in + (o & ~3u)) : (const void *)g_zero64p;
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(st + q * 1024), 16, 0, 0);
        }
        const unsigned char *wj = p.w + (long long)j * w_cs;
#pragma unroll
        for (int i = 0; i < KW; ++i) {
            const int q = wave + NWV * i;
            if (q >= W_PIECES) break;
            const int r = 16 * q + sub;
            const int s = ps ^ ((r >> 2) & 3);
            const int rs = (r / N) * w_ld + p.w_roff + r % N;  // source record (tap r / N, output channel r % N)
            __builtin_amdgcn_global_load_lds((glob_void *)(wj + rs * REC + (s << 4)),
                                             (lds_void *)(st + IN_B + q * 1024), 16, 0, 0);
        }
    };

    // ---- fragment addresses in stage 0 (stage 1: + STAGE): A = (halo column hx, tap row dy) of this wave's rows ----
    uint32_t a_hi[3], a_lo[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const int hy = 32 * wh + ml + d;
        const uint32_t o = lds_addr(lds) + hy * REC + (((2 * hl) ^ ((hy >> 2) & 3)) << 4) +
                           (uint32_t)(CW * wg) * HY * REC;
        a_hi[d] = o;
        a_lo[d] = o ^ 16u;
    }
    const uint32_t b_hi0 = lds_addr(lds) + IN_B + ml * REC + (((2 * hl) ^ ((ml >> 2) & 3)) << 4);

    f32x16 acc[CW];
    auto zero_acc = [&]() {
#pragma unroll
        for (int c = 0; c < CW; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    };
    zero_acc();

    // one K chunk from stage sb (byte offset 0 or STAGE): the column-tile kernel's d-major sweep (esr_conv_x3c.hip
    // compute(), NT = 1, TS = 3, CW = 3), every fragment address a base register plus an immediate
    auto compute = [&](uint32_t sb) {
        const uint32_t bh_b = b_hi0 + sb, bl_b = (b_hi0 + sb) ^ 16u;
        const uint32_t ah0 = a_hi[0] + sb, ah1 = a_hi[1] + sb, ah2 = a_hi[2] + sb;
        const uint32_t al0 = a_lo[0] + sb, al1 = a_lo[1] + sb, al2 = a_lo[2] + sb;
        f16x8 bh[2][3], bl[2][3], ah[3], al[3];
        auto ldb = [&](auto Dc) {
            constexpr int d = decltype(Dc)::value;
            sfor<0, 3>([&](auto Xc) {
                constexpr int dx = decltype(Xc)::value, t = d * 3 + dx;
                bh[d & 1][dx] = ds_read16<t * N * REC>(bh_b);
                bl[d & 1][dx] = ds_read16<t * N * REC>(bl_b);
            });
        };
        auto lda = [&](auto Sc) {
            constexpr int s = decltype(Sc)::value, d = s / NIC, ic = s % NIC, buf = s % 3;
            const uint32_t xh = d == 0 ? ah0 : d == 1 ? ah1 : ah2;
            const uint32_t xl = d == 0 ? al0 : d == 1 ? al1 : al2;
            ah[buf] = ds_read16<ic * HY * REC>(xh);
            al[buf] = ds_read16<ic * HY * REC>(xl);
        };
        ldb(std::integral_constant<int, 0>{});
        lda(std::integral_constant<int, 0>{});
        lda(std::integral_constant<int, 1>{});
        sfor<0, NSTEP>([&](auto Sc) {
            constexpr int s = decltype(Sc)::value, d = s / NIC, ic = s % NIC, buf = s % 3;
            constexpr int pd = (s - 1) / NIC, pic = (s - 1) % NIC;  // the previous step
            constexpr int after = s == 0 ? 2 : ((pic == 0 && pd + 1 < 3) ? 6 : 0) + (s + 1 < NSTEP ? 2 : 0);
            lgkm_wait2<after>(ah[buf], al[buf]);
            if constexpr (ic == 0) {  // B(d) is back too: pass its registers through an ordering point
#pragma unroll
                for (int x = 0; x < 3; ++x) asm volatile("" : "+v"(bh[d & 1][x]), "+v"(bl[d & 1][x]));
            }
            if constexpr (ic == 0 && d + 1 < 3) ldb(std::integral_constant<int, d + 1>{});
            if constexpr (s + 2 < NSTEP) lda(std::integral_constant<int, s + 2>{});
            sfor<0, 3>([&](auto Pc) {
                constexpr int pr = decltype(Pc)::value;
                sfor<0, 3>([&](auto Xc) {
                    constexpr int dx = decltype(Xc)::value, c = ic - dx;
                    if constexpr (c >= 0 && c < CW) {
                        const f16x8 &a = pr == 0 ? al[buf] : ah[buf];
                        const f16x8 &b = pr == 1 ? bl[d & 1][dx] : bh[d & 1][dx];
                        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc[c], 0, 0, 0);
                    }
                });
            });
        });
    };

    const esr_conv_out &o = p.o;
    const int HP = p.H + 2;
    bool ok = true;
    // epilogue of this wave's columns of `tile` straight from registers: acc[c][r] = channel 8 (r >> 2) + 4 hl +
    // (r & 3) of pixel row ml; swapping registers r = 4..7 of lanes 0-31 with r = 0..3 of lanes 32-63 (and 12..15 with
    // 8..11) leaves every lane with channels 8 (2 s + hl) + e in registers 8 s + e: split groups 2 s + hl, s = 0, 1
    // (esr_conv_x3.hip's direct epilogue).  No LDS and no barrier: it runs beside the partner wave's MFMAs.
    f32x16 pend[CW];
    auto epilogue = [&](int tile, int ncw) {
        const int x0 = (tile % p.tiles_x) * PC;
        const int R = (tile / p.tiles_x) * PT + 32 * wh + 1 + ml;  // tall padded row of this lane's pixel
        const int b = R / HP, y = R - b * HP - 1;
        if (R >= rows_tot || y < 0 || y >= p.H) return;
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            if (c >= ncw) break;
            f32x16 &a = pend[c];
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[8 * s2 + k]),
                                                                    __float_as_uint(a[8 * s2 + 4 + k]), false, false);
                    a[8 * s2 + k] = __uint_as_float(r[0]);
                    a[8 * s2 + 4 + k] = __uint_as_float(r[1]);
                }
            if constexpr ((DBG & 4) != 0) continue;
            const int x = x0 + CW * wg + c;
            const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
            const long long opix = ((long long)b * (o.out_h + 2) + oy + 1) * (long long)(o.out_w + 2) + ox + 1;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int ch = 8 * (2 * s2 + hl);
                if (ch >= p.cout) continue;
                float v[8], r1v[8], r2v[8];
                if (o.r1) load_group(reinterpret_cast<const unsigned char *>(o.r1) + (opix * o.r1_cp + o.r1_coff + ch) * 4, r1v);
                if (o.r2) load_group(reinterpret_cast<const unsigned char *>(o.r2) + (opix * o.r2_cp + o.r2_coff + ch) * 4, r2v);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = a[8 * s2 + e] * p.w_scale_inv + p.bias[ch + e];
                    v[e] = epi(o, v[e], o.r1 ? r1v[e] : 0.f, o.r2 ? r2v[e] : 0.f);
                }
                ok &= store_group(reinterpret_cast<unsigned char *>(o.out) + (opix * o.out_cp + o.out_coff + ch) * 4, v);
                if (o.out2)
                    store_group(reinterpret_cast<unsigned char *>(o.out2) + (opix * o.out2_cp + o.out2_coff + ch) * 4, v);
            }
        }
    };

    int tile = x3p_tile(blockIdx.x, gridDim.x, ntiles, 0);
    if (tile < 0) return;  // uniform over the workgroup
    int k = 0, j = 0, pend_tile = -1, pend_ncw = 0;
    unsigned mask = in_mask(tile);
    dma(tile, mask, 0, 0);
    for (int u = 0;; ++u) {
        wait_vm0();                    // this wave's part of unit u has landed (and its stores of unit u-1)
        __builtin_amdgcn_s_barrier();  // every wave's part has; every wave is done reading unit u-1's stage
        int ntile = tile, nj = j + 1;
        unsigned nmask = mask;
        if (nj == nchunk) {
            nj = 0;
            ntile = x3p_tile(blockIdx.x, gridDim.x, ntiles, k + 1);
            if (ntile >= 0) nmask = in_mask(ntile);
        }
        if (ntile >= 0 && (!(DBG & 1) || u == 0)) dma(ntile, nmask, nj, (u + 1) & 1);  // lands while u is computed
        const uint32_t sb = (u & 1) * STAGE;
        const int tw = min(PC, p.W - (tile % p.tiles_x) * PC);
        const int ncw = min(CW, max(0, tw - CW * wg));
        // the previous tile's stores: the first row half before its MFMAs, the second after, so each SIMD's two waves
        // (w, w + 4) take turns and one computes while the other stores
#pragma unroll 1
        for (int ph = 0; ph < 2; ++ph) {  // one call site of each (registers): wave half 0 stores, then computes
            if (ph == wh && pend_tile >= 0) {
                epilogue(pend_tile, pend_ncw);
                pend_tile = -1;
            }
            if (ph == 0 && ncw > 0 && !(DBG & 2)) compute(sb);
        }
        if (nj == 0) {  // the tile's last chunk: its stores go out during the next unit
#pragma unroll
            for (int c = 0; c < CW; ++c) pend[c] = acc[c];
            pend_tile = ncw > 0 ? tile : -1;
            pend_ncw = ncw;
            zero_acc();
            ++k;
        }
        if (ntile < 0) break;
        tile = ntile;
        mask = nmask;
        j = nj;
    }
    if (pend_tile >= 0) epilogue(pend_tile, pend_ncw);
    if (!ok && p.overflow) atomicOr(p.overflow, 1);
}

int n_cus_p() {
    static int n = 0;
    if (!n) {
        int dev = 0, v = 0;
        n = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
    }
    return n;
}

}  // namespace

// N = 32 3×3 conv on the persistent double-buffered kernel (taps_side 3 only; cout <= 32, not planar)
int x3p_launch(const X3cParams &p0, hipStream_t stream, int dbg) {
    if (p0.cout > 32 || p0.o.out_planar || p0.tap_y0 || p0.tap_x0) return ESR_EINVAL;
    X3cParams p = p0;
    const int cw = dbg >= 16 ? 2 : 3;
    dbg &= 15;
    p.tiles_x = (p.W + NG * cw - 1) / (NG * cw);
    p.tiles_y = (p.B * (p.H + 2) - 2 + PT - 1) / PT;
    const int ntiles = p.tiles_x * p.tiles_y;
    const dim3 grid((unsigned)min(ntiles, n_cus_p())), block(NTHR);
#define X3P(D) do { if (cw == 2) hipLaunchKernelGGL((conv_x3p_kernel<D, 2>), grid, block, 0, stream, p); \
                    else hipLaunchKernelGGL((conv_x3p_kernel<D, 3>), grid, block, 0, stream, p); } while (0)
#ifdef ESR_X3_EXPERIMENTS
    switch (dbg) {
    case 1: X3P(1); break;
    case 2: X3P(2); break;
    case 4: X3P(4); break;
    case 5: X3P(5); break;
    default: X3P(0);
    }
#else
    (void)dbg;
    X3P(0);
#endif
#undef X3P
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

#endif  // ESR_X3_EXPERIMENTS
