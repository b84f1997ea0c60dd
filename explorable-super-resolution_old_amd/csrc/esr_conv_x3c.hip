// esr_conv_x3c.hip — x3 (split-f16) 3×3 convolution / polyphase upconv, column-tile form.
//
// Same numerics, layouts and epilogue contract as esr_conv_x3.hip (read that header first): fp32 values carried as f16
// hi/lo pairs, each product a·b = a_hi·b_hi + a_hi·b_lo + a_lo·b_hi on v_mfma_f32_32x32x16_f16 with fp32 accumulation.
// What differs is how the work is cut, to spend fewer LDS reads and no VALU per MFMA:
//
//  * An M-tile (the 32 MFMA rows) is a COLUMN segment of 32 pixels of the tall batch image (B·(H+2) rows, halo rows
//    between images are the vertical padding).  The tall dimension is a multiple of 32 at every bench shape, so no
//    M-tile is partial; the width needs no multiple of 32 either (a tile is 16 columns; waves past the image width skip
//    their MFMAs).
//  * A workgroup (256 threads, 4 waves) owns a 32-row × 16-column output tile; wave w owns tile columns 4w..4w+3.
//    Two workgroups share a CU (one LDS stage each), so one's LDS-DMA, barriers and epilogue overlap the other's MFMAs.
//  * Column reuse: the A fragment of (halo column hx, tap row dy) is read from LDS once and feeds every output column
//    c = hx - dx of the wave (up to 3 taps), and each wave keeps the B fragments (weights) of all taps of a 32-channel
//    N-tile in registers for the whole K chunk.  Per 16-channel chunk a wave issues 36 A reads + 18 B reads per N-tile
//    for 108 MFMAs (the row-tile kernel: 1 read per MFMA at N = 32).
//  * LDS images are column-major: input record (hx, hy) at hx·34 + hy, its four 16-B slots XOR-swizzled by (hy>>2)&3
//    (applied on the DMA source address: the LDS-DMA destination is lane-linear), so a column shift is an immediate
//    offset and only the three tap rows need per-lane address registers; ds_read_b128 lane groups are conflict-free.
#include <hip/hip_runtime.h>
#include <type_traits>
#include "esr_amd.h"
#include "esr_x3c.h"

#ifdef ESR_X3_EXPERIMENTS
static void *g_x3c_stamps = nullptr;  // variant 87's stamp buffer (host side; handed to the kernel in X3cParams.y1)
#endif

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void glob_void;

constexpr int REC = 64;                          // bytes per staged record: 16 channels, split
constexpr int CT = 32;                           // tile rows = MFMA M
constexpr int CW = 4;                            // output columns per wave
constexpr int NWV = 4;                           // waves per workgroup
constexpr int NTHR = 64 * NWV;
constexpr int TWC = CW * NWV;                    // 16 output columns per tile
constexpr int HYC = CT + 2;                      // 34 halo rows
constexpr int HXC = TWC + 2;                     // 18 halo columns
constexpr int IN_RECS = HYC * HXC;               // 612
constexpr int IN_PIECES = (IN_RECS + 15) / 16;   // 39 one-KB LDS-DMA wave-instructions
constexpr int IN_B = IN_PIECES * 16 * REC;       // 39936
constexpr int KIN = (IN_PIECES + NWV - 1) / NWV; // input pieces per wave (10)
constexpr int N_XCD = 8;

__device__ __attribute__((aligned(16))) unsigned char g_zero64[64];
// DBG 32 (diagnostic build, variant 87): per-workgroup s_memrealtime stamps (100 MHz) of wave 0 — kernel start, then per
// K chunk (before its LDS-DMA issue, after its wait + barrier, after its compute), then after the epilogue — written
// by vector stores into the buffer passed in X3cParams.y1 (unused by this instantiation; X3C_NS stamps per workgroup)
// and read by tools/x3c_stamps.py.  Only their shares mean anything: the stamps' own waits forbid overlaps the real
// kernel has.
constexpr int X3C_NCH = 12, X3C_NS = 2 + 3 * X3C_NCH;  // (stamp slots of the DBG 32 build)

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

__device__ __forceinline__ float split_at(const float *buf, long long pix, int cp, int ch) {
    const _Float16 *g = reinterpret_cast<const _Float16 *>(buf + pix * cp + (ch & ~7));
    return (float)g[ch & 7] + (float)g[8 + (ch & 7)];
}

// blockIdx -> tile so that each XCD (blocks b, b+8, ... share one) walks one contiguous run of tiles; a bijection
__device__ __forceinline__ int xcd_tile(int b, int nb) {
    const int x = b % N_XCD, l = b / N_XCD, q = nb / N_XCD, r = nb % N_XCD;
    return x < r ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
}

__device__ __forceinline__ uint32_t lds_addr(const void *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// One 16-byte LDS read the compiler does not track (the caller waits with lgkm_wait); OFF is the immediate offset.
template <int OFF>
__device__ __forceinline__ f16x8 ds_read16(uint32_t a) {
    static_assert(OFF >= 0 && OFF < 65536, "ds_read offset");
    f16x8 r;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
    return r;
}

// s_waitcnt lgkmcnt(N) that the listed fragments pass through, so no use of them is scheduled before it
template <int N>
__device__ __forceinline__ void lgkm_wait2(f16x8 &a, f16x8 &b) {
    static_assert(N >= 0 && N < 16, "lgkmcnt");
    asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N));
}

template <int N, int K>
__device__ __forceinline__ void lgkm_wait_arr(f16x8 (&f)[K]) {
    static_assert(N >= 0 && N < 16, "lgkmcnt");
    asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f[0]) : "i"(N));
#pragma unroll
    for (int i = 1; i < K; ++i) asm volatile("" : "+v"(f[i]));
}

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// compile-time loop: f(std::integral_constant<int, i>) for i in [I, E)
template <int I, int E, class F>
__device__ __forceinline__ void sfor(F &&f) {
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, E>(f);
    }
}

// NT: 32-channel N-tiles (cout <= 32 * NT); TS: taps per side (3: 3×3 conv; 2: one polyphase upconv phase).
// DBG (diagnostic builds only, garbage outputs): 1 = LDS-DMA of chunk 0 only, 2 = no fragment reads / MFMAs,
// 4 = no epilogue stores.  RB: the B fragments (weights) are loaded from global memory (L1/L2) into registers
// instead of being staged in LDS: the LDS-DMA moves only the input halo tile (32-48 % fewer staged bytes).
// WR (NT = 1): at the start of each K chunk every wave copies the B fragments of all taps from LDS into registers,
// after which the weight stage is free: the next chunk's weights are LDS-DMA'd while this chunk is computed, so only
// the halo tile's transfer sits between two chunks' MFMAs (the weights are a third of the staged bytes at N = 32).
// TW: output columns per tile (16 by default); OCC: workgroups per CU the register budget is sized for (A/B: 12-column
// tiles of 3-column waves at three workgroups per CU, 48 KB of LDS each).
// HF: HR_conv0 fused with HR_conv1 (x3c_launch_hr1; the epilogue below the main loop).
template <int NT, int TS, int DBG = 0, bool RB = false, int CWV = CW, bool WR = false, int TW = TWC, int OCC = 2,
          bool HF = false>
__global__ __launch_bounds__(64 * (TW / CWV), (TW / CWV) * OCC / 4) void conv_x3c_kernel(X3cParams p) {
    constexpr int TWk = TW, HXk = TWk + 2, IN_RECSk = HYC * HXk, IN_PIECESk = (IN_RECSk + 15) / 16;
    constexpr int IN_Bk = IN_PIECESk * 16 * REC;
    static_assert(!WR || (NT == 1 && !RB), "register-resident weights: one N-tile, weights staged in LDS");
    constexpr int CWk = CWV;                               // output columns per wave
    constexpr int NW = TWk / CWk;                          // waves per workgroup
    constexpr int KINk = (IN_PIECESk + NW - 1) / NW;        // input pieces per wave
    constexpr int T = TS * TS;
    constexpr int N = 32 * NT;
    constexpr int W_RECS = T * N;
    constexpr int W_PIECES = W_RECS / 16;
    constexpr int KW = (W_PIECES + NW - 1) / NW;
    constexpr int W_B = W_RECS * REC;
    constexpr int LDS_BYTES = IN_Bk + (RB ? 0 : W_B);
    constexpr int EP_P = N + 4;                            // epilogue row pitch (floats)
    constexpr int NIC = CWk + TS - 1;                       // halo columns a wave reads (6 for 3×3)
    constexpr int NSTEP = NIC * TS;                        // A steps (halo column, tap row) per sweep
    static_assert(NW * 32 * EP_P * 4 <= LDS_BYTES, "per-wave epilogue areas fit in the (input + weight) stage");
    static_assert(OCC * LDS_BYTES <= 163840, "OCC workgroups per CU");
    __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hl = lane >> 5;
    const int ml = lane & 31;

    const int tile = p.xcd_map ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tx = tile % p.tiles_x;
    const int ty = tile / p.tiles_x;
    const int x0 = tx * TWk;             // first halo column = padded column x0; output padded columns x0+1+c
    const int r0 = ty * CT;              // first halo row (tall padded image); output tall rows r0+1+m
    const int tw = min(TWk, p.W - x0);   // valid output columns of the tile
    const int ncw = min(CWk, max(0, tw - CWk * wave));  // valid output columns of this wave
    const int rows_tot = p.B * (p.H + 2);
    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;
    const int nchunk = (p.cin + 15) >> 4;
    const unsigned char *tile_in = p.in + ((long long)r0 * rowp + x0) * pixb;
#ifdef ESR_X3_EXPERIMENTS
    unsigned long long stamps[(DBG & 32) ? X3C_NS : 1];
    auto stamp = [&](int idx) {
        if constexpr ((DBG & 32) != 0) {
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long t;
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");  // 100 MHz
            __builtin_amdgcn_sched_barrier(0);
            if (idx < X3C_NS) stamps[idx] = t;
        }
    };
    stamp(0);
#else
    auto stamp = [&](int) {};
#endif

    // ---- LDS-DMA addressing: input piece q of this wave = records 16 (wave + 4 i) .. +15, lane -> (record, slot) ----
    const int sub = lane >> 2, ps = lane & 3;
    unsigned in_off[KINk];  // byte offset from tile_in (slot included); bit 0 set = zero page; bit 1 = lo group
#pragma unroll
    for (int i = 0; i < KINk; ++i) {
        const int q = wave + NW * i;
        const int r = 16 * q + sub;
        const int hx = r / HYC, hy = r - (r / HYC) * HYC;
        const int s = ps ^ ((hy >> 2) & 3);
        const bool v = q < IN_PIECESk && r < IN_RECSk && r0 + hy < rows_tot && x0 + hx < p.W + 2;
        in_off[i] = v ? (unsigned)((hy * rowp + hx) * pixb + (s << 4)) | ((s >> 1) << 1) : 1u;
    }
    auto dma_in = [&](int j) {
        const int groups = min(16, p.cin - 16 * j) >> 3;  // 8-channel groups present in the chunk (1 or 2)
#pragma unroll
        for (int i = 0; i < KINk; ++i) {
            const int q = wave + NW * i;
            if (q >= IN_PIECESk) break;
            const unsigned o = in_off[i];
            const bool ok = !(o & 1u) && ((o >> 1) & 1u) < (unsigned)groups;
            const void *src = ok ? (const void *)(tile_in + (o & ~3u) + 64LL * j) : (const void *)g_zero64;
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(lds + q * 1024), 16, 0, 0);
        }
    };
    auto dma_w = [&](int j) {
        if constexpr (!RB) {
            const unsigned char *wj = p.w + (long long)j * (p.w_cstride ? p.w_cstride : (long long)W_B);
            const int ld = p.w_ld ? p.w_ld : N;
#pragma unroll
            for (int i = 0; i < KW; ++i) {
                const int q = wave + NW * i;
                if (q >= W_PIECES) break;
                const int r = 16 * q + sub;
                const int s = ps ^ ((r >> 2) & 3);
                const int rs = (r / N) * ld + p.w_roff + r % N;  // source record (tap r / N, output channel r % N)
                __builtin_amdgcn_global_load_lds((glob_void *)(wj + rs * REC + (s << 4)),
                                                 (lds_void *)(lds + IN_Bk + q * 1024), 16, 0, 0);
            }
        }
    };
    auto dma = [&](int j) {
        dma_in(j);
        dma_w(j);
    };

    // ---- fragment addresses: A (pixels, halo column hx, tap row dy): lane (ml, hl) reads record hx*HYC + ml + dy,
    // logical slot 2hl (hi) / 2hl+1 (lo); B (weights, tap t, N-tile nt): record t*N + nt*32 + ml ----
    uint32_t a_hi[TS], a_lo[TS];
#pragma unroll
    for (int d = 0; d < TS; ++d) {
        const int dy = p.tap_y0 + d;
        const int hy = ml + dy;
        const uint32_t o = lds_addr(lds) + hy * REC + (((2 * hl) ^ ((hy >> 2) & 3)) << 4) +
                           (uint32_t)(CWk * wave + p.tap_x0) * HYC * REC;
        a_hi[d] = o;
        a_lo[d] = o ^ 16u;
    }
    const uint32_t b_hi = lds_addr(lds) + IN_Bk + ml * REC + (((2 * hl) ^ ((ml >> 2) & 3)) << 4);
    const uint32_t b_lo = b_hi ^ 16u;
    const f16x8 *w_lane = reinterpret_cast<const f16x8 *>(p.w + ml * REC + 32 * hl);  // RB: this lane's B slice

    f16x8 bregh[WR ? T : 1], bregl[WR ? T : 1];  // WR: this chunk's B fragments of every tap
    f32x16 acc[CWk][NT];
#pragma unroll
    for (int c = 0; c < CWk; ++c)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[c][nt][r] = 0.f;

    // One K chunk from the staged LDS images.  Per N-tile, a sweep over steps s = (tap row d, halo column ic),
    // d-major: the A pair of step s is read two steps ahead and feeds the output columns c = ic - dx (taps (d, dx));
    // only the B fragments of tap row d are live (double-buffered: row d+1 is read at the first step of row d).  All
    // indices are compile-time, so every fragment address is a base register plus an immediate offset.  Issue order:
    // B(0), A(0), A(1), then per step s (after its wait) B(d+1) if ic == 0, and A(s+2); LDS reads complete in order,
    // so the wait for A(s) counts the reads issued after it, and B(d) (issued before A(d*NIC - NIC + 2)) is back by
    // the first step of row d.
    auto compute = [&](int j) {
        const f16x8 *wj = w_lane + (long long)j * (W_B / 16);
        sfor<0, NT>([&](auto NTc) {
            constexpr int nt = decltype(NTc)::value;
            f16x8 bh[2][TS], bl[2][TS], ah[3], al[3];
            auto ldb = [&](auto Dc) {
                constexpr int d = decltype(Dc)::value;
                if constexpr (WR) return;
                sfor<0, TS>([&](auto Xc) {
                    constexpr int dx = decltype(Xc)::value, t = d * TS + dx;
                    if constexpr ((DBG & 16) != 0) {
                        bh[d & 1][dx] = f16x8{};
                        bl[d & 1][dx] = f16x8{};
                        asm volatile("" : "+v"(bh[d & 1][dx]), "+v"(bl[d & 1][dx]));
                    } else if constexpr (RB) {  // global (L1/L2) loads; the compiler waits for them before first use
                        bh[d & 1][dx] = wj[(t * N + nt * 32) * (REC / 16)];
                        bl[d & 1][dx] = wj[(t * N + nt * 32) * (REC / 16) + 1];
                    } else {
                        bh[d & 1][dx] = ds_read16<(t * N + nt * 32) * REC>(b_hi);
                        bl[d & 1][dx] = ds_read16<(t * N + nt * 32) * REC>(b_lo);
                    }
                });
            };
            auto lda = [&](auto Sc) {
                constexpr int s = decltype(Sc)::value, d = s / NIC, ic = s % NIC, buf = s % 3;
                if constexpr ((DBG & 16) != 0) {  // diagnostic: no fragment reads (operands from the registers)
                    ah[buf] = bh[0][0];
                    al[buf] = bl[0][0];
                    return;
                }
                ah[buf] = ds_read16<ic * HYC * REC>(a_hi[d]);
                al[buf] = ds_read16<ic * HYC * REC>(a_lo[d]);
            };
            ldb(std::integral_constant<int, 0>{});
            lda(std::integral_constant<int, 0>{});
            if constexpr (NSTEP > 1) lda(std::integral_constant<int, 1>{});
            sfor<0, NSTEP>([&](auto Sc) {
                constexpr int s = decltype(Sc)::value, d = s / NIC, ic = s % NIC, buf = s % 3;
                constexpr int pd = (s - 1) / NIC, pic = (s - 1) % NIC;  // the previous step
                constexpr int after = s == 0 ? (NSTEP > 1 ? 2 : 0)
                                             : ((!RB && !WR && pic == 0 && pd + 1 < TS) ? 2 * TS : 0) +
                                               (s + 1 < NSTEP ? 2 : 0);
                lgkm_wait2<after>(ah[buf], al[buf]);
                if constexpr (ic == 0 && !RB && !WR) {  // B(d) is back too: pass its registers through an ordering point
#pragma unroll
                    for (int x = 0; x < TS; ++x) asm volatile("" : "+v"(bh[d & 1][x]), "+v"(bl[d & 1][x]));
                }
                if constexpr (ic == 0 && d + 1 < TS) ldb(std::integral_constant<int, d + 1>{});
                if constexpr (s + 2 < NSTEP) lda(std::integral_constant<int, s + 2>{});
                // products lo*hi, hi*lo, hi*hi, each over the output columns c = ic - dx this A pair feeds
                sfor<0, 3>([&](auto Pc) {
                    constexpr int pr = decltype(Pc)::value;
                    sfor<0, TS>([&](auto Xc) {
                        constexpr int dx = decltype(Xc)::value, c = ic - dx;
                        if constexpr (c >= 0 && c < CWk && !(DBG & 8)) {  // DBG 8: the reads without the MFMAs
                            const f16x8 &a = pr == 0 ? al[buf] : ah[buf];
                            const f16x8 &b = WR ? (pr == 1 ? bregl[WR ? d * TS + dx : 0] : bregh[WR ? d * TS + dx : 0])
                                                : (pr == 1 ? bl[d & 1][dx] : bh[d & 1][dx]);
                            acc[c][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[c][nt], 0, 0, 0);
                        }
                    });
                });
            });
        });
    };

    if constexpr (WR) {
        dma(0);
        for (int j = 0; j < nchunk; ++j) {
            wait_vm0();
            __builtin_amdgcn_s_barrier();  // chunk j's halo and weights have landed for every wave
            sfor<0, T>([&](auto Tc) {
                constexpr int t = decltype(Tc)::value;
                bregh[t] = ds_read16<t * N * REC>(b_hi);
                bregl[t] = ds_read16<t * N * REC>(b_lo);
            });
            lgkm_wait_arr<0>(bregh);
#pragma unroll
            for (int t = 0; t < T; ++t) asm volatile("" : "+v"(bregl[t]));
            __builtin_amdgcn_s_barrier();  // every wave holds its B fragments: the weight stage is free
            if (j + 1 < nchunk) dma_w(j + 1);  // lands while chunk j is computed
            if (ncw > 0) compute(j);
            if (j + 1 < nchunk) {
                __builtin_amdgcn_s_barrier();  // every wave is done reading the halo stage
                dma_in(j + 1);
            }
        }
    } else {
    for (int j = 0; j < nchunk; ++j) {
        if (j) __builtin_amdgcn_s_barrier();  // every wave is done reading the stage (its reads were waited for)
        if ((DBG & 32) && j < X3C_NCH) stamp(1 + 3 * j);
        if (!(DBG & 1) || j == 0) dma(j);
        wait_vm0();
        __builtin_amdgcn_s_barrier();
        if ((DBG & 32) && j < X3C_NCH) stamp(2 + 3 * j);
        if (ncw > 0 && !(DBG & 2)) compute(j);
        if ((DBG & 32) && j < X3C_NCH) stamp(3 + 3 * j);
    }
    }

    // ---- epilogue: each wave restages one output column at a time through its own LDS area and stores it ----
    __builtin_amdgcn_s_barrier();  // all waves are done with the input (and weight) stage it aliases
    if (ncw <= 0) return;
    const esr_conv_out &o = p.o;
    float *s_ep = reinterpret_cast<float *>(lds) + wave * 32 * EP_P;
    constexpr int G = N / 8;            // 8-channel groups per pixel
    constexpr int ITEMS = 32 * G / 64;  // (pixel, group) items per lane per column
    const int HP = p.H + 2;
    bool ok = true;
    if constexpr (HF) {
        // HR_conv0 (+ LeakyReLU) -> HR_conv1 (architecture.py:140-141) without storing HR_conv0's activations: per
        // pixel, Y[3t + o] = Σ_c W1[o][c][t] · a[c] over HR_conv1's input channels c = [latent slot | activations]
        // (t = its 3×3 tap, o = its output channel), on the x3 MFMA with the pixels in M (32 per column, lane row ml)
        // and the 27 (t, o) pairs in N (of 32); esr_hr1_sum then adds Y over each output pixel's 3×3 neighbours.  The
        // A operand is split from the fp32 activation exactly as store_group would have stored it (and flagged), the
        // latent slot is read split from the input (prep_hr wrote it there), B = HR_conv1's x3-packed weights.
        static_assert(NT == 2 && TS == 3 && !RB && !WR, "fused HR_conv1: HR_conv0 is a 3x3 N = 64 conv");
        const int zc = p.zc1, nks = (zc + 64 + 15) >> 4;
        const int n1 = ml < 27 ? ml : 0, t1 = n1 / 3, o1 = n1 - 3 * t1;
#pragma unroll
        for (int c = 0; c < CWk; ++c) {
            if (c >= ncw) break;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = 8 * (r >> 2) + 4 * hl + (r & 3);
                    s_ep[m * EP_P + nt * 32 + ml] = acc[c][nt][r];
                }
            const int x = x0 + CWk * wave + c;  // interior column; padded column x + 1
            const int R = r0 + 1 + ml;          // this lane's A row: tall padded row of pixel m = ml
            const int yb = R - (R / HP) * HP - 1;
            const bool pv = R < rows_tot && yb >= 0 && yb < p.H;
            const long long pix = (long long)R * rowp + x + 1;
            f32x16 y = {};
            for (int ks = 0; ks < nks; ++ks) {
                const int bc = 16 * ks + 8 * hl;  // first channel of this lane's 8-channel group (HR_conv1's input)
                f16x8 ah = {}, al = {}, bh = {}, bl = {};
                if (pv && bc < zc) {
                    const unsigned char *zp = p.in + pix * pixb + 4LL * bc;
                    ah = *reinterpret_cast<const f16x8 *>(zp);
                    al = *reinterpret_cast<const f16x8 *>(zp + 16);
                } else if (pv && bc - zc < 64) {
                    const int f = bc - zc;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float v = lrelu(s_ep[ml * EP_P + f + e] * p.w_scale_inv + p.bias[f + e]);
                        ah[e] = (_Float16)v;
                        al[e] = (_Float16)(v - (float)ah[e]);
                        ok = ok && (fabsf(v) < 65504.f);
                    }
                }
                if (ml < 27) {
                    const unsigned char *wp = p.w1 + ((long long)(ks * 9 + t1) * 32 + o1) * REC + 32 * hl;
                    bh = *reinterpret_cast<const f16x8 *>(wp);
                    bl = *reinterpret_cast<const f16x8 *>(wp + 16);
                }
                y = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, y, 0, 0, 0);
                y = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, y, 0, 0, 0);
                y = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, y, 0, 0, 0);
            }
            // lane (ml, hl) holds Y[m][n = ml] for m = 8(r>>2) + 4hl + (r&3): 32 lanes store one pixel's 128-B record
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = 8 * (r >> 2) + 4 * hl + (r & 3);
                const int Rm = r0 + 1 + m;
                const int ym = Rm - (Rm / HP) * HP - 1;
                if (Rm < rows_tot && ym >= 0 && ym < p.H) p.y1[((long long)Rm * rowp + x + 1) * 32 + ml] = y[r];
            }
        }
        if (!ok && p.overflow) atomicOr(p.overflow, 1);
        return;
    }
    float bk[ITEMS][8];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const int g = (lane + 64 * k) % G;
#pragma unroll
        for (int e = 0; e < 8; ++e) bk[k][e] = (8 * g + e < p.cout) ? p.bias[8 * g + e] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < CWk; ++c) {
        if (c >= ncw) break;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = 8 * (r >> 2) + 4 * hl + (r & 3);
                s_ep[m * EP_P + nt * 32 + ml] = acc[c][nt][r];
            }
        const int x = x0 + CWk * wave + c;  // interior column of the output pixel
        if constexpr ((DBG & 4) != 0) continue;  // diagnostic: restage only, no global loads / stores
        if (o.out_planar) {
            for (int it = lane; it < 32 * p.cout; it += 64) {
                const int ch = it / 32, m = it % 32;
                const int R = r0 + 1 + m;
                const int b = R / HP, y = R - b * HP - 1;
                if (R >= rows_tot || y < 0 || y >= p.H) continue;
                const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
                const long long opix = ((long long)b * (o.out_h + 2) + oy + 1) * (long long)(o.out_w + 2) + ox + 1;
                float v = s_ep[m * EP_P + ch] * p.w_scale_inv + p.bias[ch];
                v = epi(o, v, o.r1 ? split_at(o.r1, opix, o.r1_cp, o.r1_coff + ch) : 0.f, o.r2 ? split_at(o.r2, opix, o.r2_cp, o.r2_coff + ch) : 0.f);
                o.out[(((long long)b * p.cout + ch) * o.out_h + oy) * o.out_w + ox] = v;
            }
        } else {
            long long opix[ITEMS];
            bool val[ITEMS];
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                const int it = lane + 64 * k, m = it / G, g = it % G;
                const int R = r0 + 1 + m;
                const int b = R / HP, y = R - b * HP - 1;
                const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
                opix[k] = ((long long)b * (o.out_h + 2) + oy + 1) * (long long)(o.out_w + 2) + ox + 1;
                val[k] = R < rows_tot && y >= 0 && y < p.H && 8 * g < p.cout;
            }
            float r1v[ITEMS][8], r2v[ITEMS][8];
            if (o.r1) {
#pragma unroll
                for (int k = 0; k < ITEMS; ++k)
                    if (val[k])
                        load_group(reinterpret_cast<const unsigned char *>(o.r1) +
                                       (opix[k] * o.r1_cp + o.r1_coff + 8 * ((lane + 64 * k) % G)) * 4, r1v[k]);
            }
            if (o.r2) {
#pragma unroll
                for (int k = 0; k < ITEMS; ++k)
                    if (val[k])
                        load_group(reinterpret_cast<const unsigned char *>(o.r2) +
                                       (opix[k] * o.r2_cp + o.r2_coff + 8 * ((lane + 64 * k) % G)) * 4, r2v[k]);
            }
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                if (!val[k]) continue;
                const int it = lane + 64 * k, m = it / G, g = it % G;
                float v[8];
                const f32x4 v0 = *reinterpret_cast<const f32x4 *>(s_ep + m * EP_P + 8 * g);
                const f32x4 v1 = *reinterpret_cast<const f32x4 *>(s_ep + m * EP_P + 8 * g + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) { v[e] = v0[e]; v[e + 4] = v1[e]; }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = v[e] * p.w_scale_inv + bk[k][e];
                    v[e] = epi(o, v[e], o.r1 ? r1v[k][e] : 0.f, o.r2 ? r2v[k][e] : 0.f);
                }
                ok &= store_group(reinterpret_cast<unsigned char *>(o.out) + (opix[k] * o.out_cp + o.out_coff + 8 * g) * 4, v);
                if (o.out2)
                    store_group(reinterpret_cast<unsigned char *>(o.out2) + (opix[k] * o.out2_cp + o.out2_coff + 8 * g) * 4, v);
            }
        }
    }
    if (!ok && p.overflow) atomicOr(p.overflow, 1);
#ifdef ESR_X3_EXPERIMENTS
    if constexpr ((DBG & 32) != 0) {
        stamp(X3C_NS - 1);
        unsigned long long *sp = reinterpret_cast<unsigned long long *>(p.y1);
        if (wave == 0 && lane == 0 && sp) {
            for (int i = 0; i < X3C_NS; ++i) sp[(long long)blockIdx.x * X3C_NS + i] = stamps[i];
        }
    }
#endif
}

#ifdef ESR_X3_EXPERIMENTS  // measured 4-12 % slower than the one-stage kernel (profiles/r5_x3d_ab.txt): ablation only
// ---- 8-channel double-buffered form (x3d): N = 32 3×3 convs ------------------------------------------------------
// The 12-column tile of four 3-column waves at three workgroups per CU (as conv_x3c_kernel<1, 3, 0, false, 3, false,
// 12, 3>), but its K loop runs over 8-channel chunks in TWO LDS stages of 24 KB (the one-stage kernel's 48 KB): chunk
// k+1's halo and weights are LDS-DMA'd while chunk k is computed, so a workgroup no longer alternates between waiting
// for its loads and computing (stamped build, tools/x3c_stamps.py: 3.5 µs load wait + 2.7 µs compute per 16-channel
// chunk at config 2).  A staged record is one pixel's (or one weight row's) 8 channels, split: [hi 8 | lo 8], 32 B
// (the global split layout's 8-channel group).  With K = 8 channels the three products a·b = a_hi·b_hi + a_hi·b_lo +
// a_lo·b_hi go on the K = 16 MFMA as
//   cross terms  [a_lo | a_hi] · [b_hi ; b_lo]                 one MFMA per tap (9);
//   hi·hi        [a_hi(col c) | a_hi(col c+1)] · [b_hi(d,0) ; b_hi(d,1)]  per tap row d (3), the taps (d,0) + (d,1);
//                [a_hi(row 0) | a_hi(row 1)] · [b_hi(0,2) ; b_hi(1,2)]    at tap column 2 (1);
//                [a_lo | a_hi] · [0 ; b_hi(2,2)]                           the last tap (1);
// 14 MFMAs per output column and chunk (13.5 for the three products of 72 channel-taps: 3.7 % padding).  The same
// products as the one-stage kernel, summed in another order (not bitwise equal to it; same fp32-level accuracy).
// LDS images: column-major records as conv_x3c (halo record (hx, hy) at hx·34 + hy, weight record (t, n) at t·32 + n);
// the two 16-B slots of a record are swapped when bit 3 of its row is set, which makes every ds_read_b128 lane group
// conflict-free (rows m and m + 8 share a bank quad otherwise).
constexpr int XD_REC = 32, XD_HX = 14, XD_HY = 34;
constexpr int XD_IN_RECS = XD_HX * XD_HY;             // 476
constexpr int XD_IN_PIECES = (XD_IN_RECS + 31) / 32;  // 15 one-KB LDS-DMA wave-instructions (32 records each)
constexpr int XD_IN_B = XD_IN_PIECES * 1024;          // 15360
constexpr int XD_W_PIECES = 9 * 32 / 32;              // 9
constexpr int XD_STAGE = XD_IN_B + XD_W_PIECES * 1024;  // 24576
constexpr int XD_PIECES = XD_IN_PIECES + XD_W_PIECES;   // 24
constexpr int XD_NW = 4, XD_CW = 3, XD_KP = XD_PIECES / XD_NW;  // 6 pieces per wave and chunk
static_assert(XD_PIECES % XD_NW == 0, "pieces per wave");
static_assert(XD_NW * 32 * (32 + 4) * 4 <= 2 * XD_STAGE, "epilogue restage areas fit");

__device__ __forceinline__ int xd_sw(int row) { return (row >> 3) & 1; }

// one 16-byte LDS read at a run-time address (the caller waits with lgkm_wait)
__device__ __forceinline__ f16x8 ds_read16_at(uint32_t a) {
    f16x8 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
    return r;
}

__global__ __launch_bounds__(256, 3) void conv_x3d_kernel(X3cParams p) {
    __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * XD_STAGE];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hl = lane >> 5;
    const int ml = lane & 31;
    const int tile = p.xcd_map ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const int tx = tile % p.tiles_x;
    const int ty = tile / p.tiles_x;
    const int x0 = tx * 12;
    const int r0 = ty * CT;
    const int tw = min(12, p.W - x0);
    const int ncw = min(XD_CW, max(0, tw - XD_CW * wave));
    const int rows_tot = p.B * (p.H + 2);
    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;
    const int nk = p.cin >> 3;  // 8-channel chunks
    const unsigned char *tile_in = p.in + ((long long)r0 * rowp + x0) * pixb;
    const int ld = p.w_ld ? p.w_ld : 32;
    const long long wcs = p.w_cstride ? p.w_cstride : 9LL * 32 * 64;  // bytes per 16-channel chunk of the packing

    // LDS-DMA sources of this lane: piece q = wave + 4 i -> LDS record 32 q + lane / 2, physical slot lane & 1
    unsigned src_off[XD_KP];  // halo: byte offset from tile_in (bit 0: zero page); weights: offset in a 16-ch chunk
#pragma unroll
    for (int i = 0; i < XD_KP; ++i) {
        const int q = wave + XD_NW * i;
        const int ps = lane & 1;
        if (q < XD_IN_PIECES) {
            const int r = 32 * q + (lane >> 1);
            const int hx = r / XD_HY, hy = r - (r / XD_HY) * XD_HY;
            const int s = ps ^ xd_sw(hy);
            const bool v = r < XD_IN_RECS && r0 + hy < rows_tot && x0 + hx < p.W + 2;
            src_off[i] = v ? (unsigned)((hy * rowp + hx) * pixb + 16 * s) : 1u;
        } else {
            const int rw = 32 * (q - XD_IN_PIECES) + (lane >> 1);
            const int t = rw >> 5, n = rw & 31;
            const int s = ps ^ xd_sw(n);
            src_off[i] = (unsigned)((t * ld + p.w_roff + n) * 64 + 16 * s);
        }
    }
    auto dma = [&](int k, int stg) {
        unsigned char *base = lds + stg * XD_STAGE;
        const unsigned char *wk = p.w + (long long)(k >> 1) * wcs + 32 * (k & 1);
#pragma unroll
        for (int i = 0; i < XD_KP; ++i) {
            const int q = wave + XD_NW * i;
            const unsigned o = src_off[i];
            const void *src = q < XD_IN_PIECES ? ((o & 1u) ? (const void *)g_zero64 : (const void *)(tile_in + o + 32LL * k))
                                                : (const void *)(wk + o);
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(base + q * 1024), 16, 0, 0);
        }
    };

    f32x16 acc[XD_CW];
#pragma unroll
    for (int c = 0; c < XD_CW; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;

    // fragment addresses (bytes, relative to a stage): halo record (hx, hy) of this wave's columns, weight record (t, n)
    const int hb = XD_CW * wave * XD_HY;  // first halo record of this wave's columns
    auto a_at = [&](int ic, int row, int slot) {
        return (uint32_t)((hb + ic * XD_HY + row) * XD_REC + 16 * (slot ^ xd_sw(row)));
    };
    auto b_at = [&](int t, int slot) { return (uint32_t)(XD_IN_B + (t * 32 + ml) * XD_REC + 16 * (slot ^ xd_sw(ml))); };

    auto compute = [&](int stg) {
        const uint32_t sb = lds_addr(lds) + stg * XD_STAGE;
        f16x8 zero = {};
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            // tap row d: cross-term A of the 5 halo columns, the hi-pair A of the 3 output columns, its weights
            f16x8 ax[XD_CW + 2], ap[XD_CW], bx[3], bp, bs;
#pragma unroll
            for (int ic = 0; ic < XD_CW + 2; ++ic) ax[ic] = ds_read16_at(sb + a_at(ic, ml + d, 1 - hl));
#pragma unroll
            for (int c = 0; c < XD_CW; ++c) ap[c] = ds_read16_at(sb + a_at(c + hl, ml + d, 0));
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) bx[dx] = ds_read16_at(sb + b_at(3 * d + dx, hl));
            bp = ds_read16_at(sb + b_at(3 * d + hl, 0));
            if (d == 2) bs = ds_read16_at(sb + b_at(8, 0));
            lgkm_wait_arr<0>(ax);
#pragma unroll
            for (int c = 0; c < XD_CW; ++c) asm volatile("" : "+v"(ap[c]));
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) asm volatile("" : "+v"(bx[dx]));
            asm volatile("" : "+v"(bp));
            if (d == 2) {
                asm volatile("" : "+v"(bs));
                if (!hl) bs = zero;
            }
#pragma unroll
            for (int ic = 0; ic < XD_CW + 2; ++ic)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    const int c = ic - dx;
                    if (c >= 0 && c < XD_CW) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[ic], bx[dx], acc[c], 0, 0, 0);
                }
#pragma unroll
            for (int c = 0; c < XD_CW; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ap[c], bp, acc[c], 0, 0, 0);
            if (d == 2) {
#pragma unroll
                for (int c = 0; c < XD_CW; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ax[c + 2], bs, acc[c], 0, 0, 0);
            }
        }
        // tap column 2, rows 0 and 1: [a_hi(row 0) | a_hi(row 1)] · [b_hi(0,2) ; b_hi(1,2)]
        f16x8 ar[XD_CW], br;
#pragma unroll
        for (int c = 0; c < XD_CW; ++c) ar[c] = ds_read16_at(sb + a_at(c + 2, ml + hl, 0));
        br = ds_read16_at(sb + b_at(2 + 3 * hl, 0));
        lgkm_wait_arr<0>(ar);
        asm volatile("" : "+v"(br));
#pragma unroll
        for (int c = 0; c < XD_CW; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ar[c], br, acc[c], 0, 0, 0);
    };

    if (nk > 0) dma(0, 0);
    for (int k = 0; k < nk; ++k) {
        wait_vm0();                    // this wave's pieces of chunk k have landed
        __builtin_amdgcn_s_barrier();  // ... every wave's; and every wave is done with chunk k - 1's stage
        if (k + 1 < nk) dma(k + 1, (k + 1) & 1);
        if (ncw > 0) compute(k & 1);
    }

    // ---- epilogue (as conv_x3c_kernel's): each wave restages one output column at a time through its own LDS area
    __builtin_amdgcn_s_barrier();
    if (ncw <= 0) return;
    constexpr int N = 32, EP_P = N + 4, CWk = XD_CW, NT = 1;
    const esr_conv_out &o = p.o;
    float *s_ep = reinterpret_cast<float *>(lds) + wave * 32 * EP_P;
    constexpr int G = N / 8;
    constexpr int ITEMS = 32 * G / 64;
    const int HP = p.H + 2;
    bool ok = true;
    float bk[ITEMS][8];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const int g = (lane + 64 * k) % G;
#pragma unroll
        for (int e = 0; e < 8; ++e) bk[k][e] = (8 * g + e < p.cout) ? p.bias[8 * g + e] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < CWk; ++c) {
        if (c >= ncw) break;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = 8 * (r >> 2) + 4 * hl + (r & 3);
            s_ep[m * EP_P + ml] = acc[c][r];
        }
        const int x = x0 + CWk * wave + c;  // interior column of the output pixel
        if (o.out_planar) {
            for (int it = lane; it < 32 * p.cout; it += 64) {
                const int ch = it / 32, m = it % 32;
                const int R = r0 + 1 + m;
                const int b = R / HP, y = R - b * HP - 1;
                if (R >= rows_tot || y < 0 || y >= p.H) continue;
                const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
                const long long opix = ((long long)b * (o.out_h + 2) + oy + 1) * (long long)(o.out_w + 2) + ox + 1;
                float v = s_ep[m * EP_P + ch] * p.w_scale_inv + p.bias[ch];
                v = epi(o, v, o.r1 ? split_at(o.r1, opix, o.r1_cp, o.r1_coff + ch) : 0.f, o.r2 ? split_at(o.r2, opix, o.r2_cp, o.r2_coff + ch) : 0.f);
                o.out[(((long long)b * p.cout + ch) * o.out_h + oy) * o.out_w + ox] = v;
            }
        } else {
            long long opix[ITEMS];
            bool val[ITEMS];
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                const int it = lane + 64 * k, m = it / G, g = it % G;
                const int R = r0 + 1 + m;
                const int b = R / HP, y = R - b * HP - 1;
                const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
                opix[k] = ((long long)b * (o.out_h + 2) + oy + 1) * (long long)(o.out_w + 2) + ox + 1;
                val[k] = R < rows_tot && y >= 0 && y < p.H && 8 * g < p.cout;
            }
            float r1v[ITEMS][8], r2v[ITEMS][8];
            if (o.r1) {
#pragma unroll
                for (int k = 0; k < ITEMS; ++k)
                    if (val[k])
                        load_group(reinterpret_cast<const unsigned char *>(o.r1) +
                                       (opix[k] * o.r1_cp + o.r1_coff + 8 * ((lane + 64 * k) % G)) * 4, r1v[k]);
            }
            if (o.r2) {
#pragma unroll
                for (int k = 0; k < ITEMS; ++k)
                    if (val[k])
                        load_group(reinterpret_cast<const unsigned char *>(o.r2) +
                                       (opix[k] * o.r2_cp + o.r2_coff + 8 * ((lane + 64 * k) % G)) * 4, r2v[k]);
            }
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                if (!val[k]) continue;
                const int it = lane + 64 * k, m = it / G, g = it % G;
                float v[8];
                const f32x4 v0 = *reinterpret_cast<const f32x4 *>(s_ep + m * EP_P + 8 * g);
                const f32x4 v1 = *reinterpret_cast<const f32x4 *>(s_ep + m * EP_P + 8 * g + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) { v[e] = v0[e]; v[e + 4] = v1[e]; }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    v[e] = v[e] * p.w_scale_inv + bk[k][e];
                    v[e] = epi(o, v[e], o.r1 ? r1v[k][e] : 0.f, o.r2 ? r2v[k][e] : 0.f);
                }
                ok &= store_group(reinterpret_cast<unsigned char *>(o.out) + (opix[k] * o.out_cp + o.out_coff + 8 * g) * 4, v);
                if (o.out2)
                    store_group(reinterpret_cast<unsigned char *>(o.out2) + (opix[k] * o.out2_cp + o.out2_coff + 8 * g) * 4, v);
            }
        }
    }
    if (!ok && p.overflow) atomicOr(p.overflow, 1);
    (void)NT;
}

#endif  // ESR_X3_EXPERIMENTS (x3d)

#ifdef ESR_X3_EXPERIMENTS  // spills at its register budget and runs 2-5x slower (r2 A/B): experiment library only
// ---- warp-specialised persistent form --------------------------------------------------------------------------
//
// One workgroup per CU walks its tiles (an XCD-local band, x3s_tile) as one stream of units u = (tile, K chunk).
// Compute waves own 4 output columns and one 32-channel N-tile each (N = 64: 8 compute waves, two per SIMD; N = 32:
// 4); the last 4 waves only move data: they stage unit u+1 into the other LDS stage by LDS-DMA while unit u is
// computed, so the matrix pipes never wait for a tile's loads, not even at tile boundaries.  One s_barrier per unit:
// [loaders: DMA(u+1), vmcnt(0) | compute waves: unit u, their last LDS read waited] -> barrier.  The MFMA operands
// are swapped (weights as A, pixels as B), so each lane ends with channels of ONE pixel and the epilogue
// (v_permlane32_swap regroup, bias, LeakyReLU, residuals, split, 16-B stores) runs from registers: no LDS restage,
// and the loaders keep both stages busy across it.
constexpr int S_CW = 4;                               // output columns per compute wave
constexpr int S_NLW = 4;                              // loader waves
static_assert(S_CW * 4 == TWC, "four compute waves span the tile width");
constexpr int S_KIN = (IN_PIECES + S_NLW - 1) / S_NLW;

// k-th tile of workgroup b in a grid of g: XCD x = b % 8 owns tiles [x Q, (x+1) Q) (Q = ceil(ntiles / 8)), dealt
// round-robin to its workgroups, so the tiles in flight on one XCD are neighbours (their halos share its L2).  -1 past
// the end.
__device__ __forceinline__ int x3s_tile(int b, int g, int ntiles, int k) {
    const int x = b % N_XCD, l = b / N_XCD;
    const int per = (g - x + N_XCD - 1) / N_XCD;  // workgroups on XCD x
    const int q = (ntiles + N_XCD - 1) / N_XCD;
    const int t = l + k * per;
    return (t < q && x * q + t < ntiles) ? x * q + t : -1;
}

template <int NT> struct X3sShape {
    static constexpr int NCOMP = 4 * NT;                  // compute waves
    static constexpr int NTHR = 64 * (NCOMP + S_NLW);
    static constexpr int WPS = (NCOMP + S_NLW) / 4;       // waves per SIMD (register budget 512 / WPS)
};

template <int NT, int TS, int DBG = 0>
__global__ __launch_bounds__(X3sShape<NT>::NTHR, X3sShape<NT>::WPS) void conv_x3s_kernel(X3cParams p) {
    constexpr int NCOMP = X3sShape<NT>::NCOMP;
    constexpr int T = TS * TS;
    constexpr int N = 32 * NT;
    constexpr int W_RECS = T * N;
    constexpr int W_PIECES = W_RECS / 16;
    constexpr int KW = (W_PIECES + S_NLW - 1) / S_NLW;
    constexpr int W_B = W_RECS * REC;
    constexpr int STAGE = IN_B + W_B;
    constexpr int NIC = S_CW + TS - 1;
    constexpr int NSTEP = NIC * TS;
    static_assert(2 * STAGE <= 163840, "two LDS stages");
    __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool is_loader = wave >= NCOMP;
    const int cw = wave & 3;        // compute wave: column group
    const int nt = wave >> 2;       // compute wave: N-tile
    const int hl = lane >> 5;
    const int ml = lane & 31;
    const int ntiles = p.tiles_x * p.tiles_y;
    const int rows_tot = p.B * (p.H + 2);
    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;
    const int nchunk = (p.cin + 15) >> 4;
    int ntile_mine = 0;
    while (x3s_tile(blockIdx.x, gridDim.x, ntiles, ntile_mine) >= 0) ++ntile_mine;
    const int nunits = ntile_mine * nchunk;

    // ---- loader side: no state across units (addresses recomputed per unit) ----
    auto dma = [&](int u) {
        const int lw = wave - NCOMP;
        const int sub = lane >> 2, ps = lane & 3;
        const int k = u / nchunk, j = u - k * nchunk;
        const int t = x3s_tile(blockIdx.x, gridDim.x, ntiles, k);
        const int x0 = (t % p.tiles_x) * TWC, r0 = (t / p.tiles_x) * CT;
        const unsigned char *tile_in = p.in + ((long long)r0 * rowp + x0) * pixb + 64LL * j;
        unsigned char *st = lds + (u & 1) * STAGE;
        const int groups = min(16, p.cin - 16 * j) >> 3;
#pragma unroll
        for (int i = 0; i < S_KIN; ++i) {
            const int q = lw + S_NLW * i;
            if (q >= IN_PIECES) break;
            const int r = 16 * q + sub;
            const int hx = r / HYC, hy = r - (r / HYC) * HYC;
            const int s = ps ^ ((hy >> 2) & 3);
            const bool ok = r < IN_RECS && r0 + hy < rows_tot && x0 + hx < p.W + 2 && (s >> 1) < groups;
            const void *src = ok ? (const void *)(tile_in + (hy * rowp + hx) * pixb + (s << 4)) : (const void *)g_zero64;
            __builtin_amdgcn_global_load_lds((glob_void *)src, (lds_void *)(st + q * 1024), 16, 0, 0);
        }
        const unsigned char *wj = p.w + (long long)j * W_B;
#pragma unroll
        for (int i = 0; i < KW; ++i) {
            const int q = lw + S_NLW * i;
            if (q >= W_PIECES) break;
            const int r = 16 * q + sub;
            const int s = ps ^ ((r >> 2) & 3);
            __builtin_amdgcn_global_load_lds((glob_void *)(wj + r * REC + (s << 4)),
                                             (lds_void *)(st + IN_B + q * 1024), 16, 0, 0);
        }
    };

    // ---- compute side: fragment base addresses in stage 0 (stage 1: + STAGE) ----
    uint32_t a_hi[TS], a_lo[TS];
#pragma unroll
    for (int d = 0; d < TS; ++d) {
        const int hy = ml + p.tap_y0 + d;
        const uint32_t o = lds_addr(lds) + hy * REC + (((2 * hl) ^ ((hy >> 2) & 3)) << 4) +
                           (uint32_t)(S_CW * cw + p.tap_x0) * HYC * REC;
        a_hi[d] = o;
        a_lo[d] = o ^ 16u;
    }
    const uint32_t b_hi0 = lds_addr(lds) + IN_B + (nt * 32 + ml) * REC + (((2 * hl) ^ ((ml >> 2) & 3)) << 4);

    f32x16 acc[S_CW];
    auto zero_acc = [&]() {
#pragma unroll
        for (int c = 0; c < S_CW; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    };
    zero_acc();

    // one unit from stage sb (0 or STAGE bytes): the d-major sweep of conv_x3c_kernel for this wave's N-tile, with
    // swapped MFMA operands
    auto compute = [&](uint32_t sb) {
        const uint32_t bh_b = b_hi0 + sb, bl_b = (b_hi0 + sb) ^ 16u;
        f16x8 bh[2][TS], bl[2][TS], ah[3], al[3];
        auto ldb = [&](auto Dc) {
            constexpr int d = decltype(Dc)::value;
            sfor<0, TS>([&](auto Xc) {
                constexpr int dx = decltype(Xc)::value, t = d * TS + dx;
                bh[d & 1][dx] = ds_read16<t * N * REC>(bh_b);
                bl[d & 1][dx] = ds_read16<t * N * REC>(bl_b);
            });
        };
        auto lda = [&](auto Sc) {
            constexpr int s = decltype(Sc)::value, d = s / NIC, ic = s % NIC, buf = s % 3;
            ah[buf] = ds_read16<ic * HYC * REC>(a_hi[d] + sb);
            al[buf] = ds_read16<ic * HYC * REC>(a_lo[d] + sb);
        };
        ldb(std::integral_constant<int, 0>{});
        lda(std::integral_constant<int, 0>{});
        if constexpr (NSTEP > 1) lda(std::integral_constant<int, 1>{});
        sfor<0, NSTEP>([&](auto Sc) {
            constexpr int s = decltype(Sc)::value, d = s / NIC, ic = s % NIC, buf = s % 3;
            constexpr int pd = (s - 1) / NIC, pic = (s - 1) % NIC;
            constexpr int after = s == 0 ? (NSTEP > 1 ? 2 : 0)
                                         : ((pic == 0 && pd + 1 < TS) ? 2 * TS : 0) + (s + 1 < NSTEP ? 2 : 0);
            lgkm_wait2<after>(ah[buf], al[buf]);
            if constexpr (ic == 0) {
#pragma unroll
                for (int x = 0; x < TS; ++x) asm volatile("" : "+v"(bh[d & 1][x]), "+v"(bl[d & 1][x]));
            }
            if constexpr (ic == 0 && d + 1 < TS) ldb(std::integral_constant<int, d + 1>{});
            if constexpr (s + 2 < NSTEP) lda(std::integral_constant<int, s + 2>{});
            sfor<0, 3>([&](auto Pc) {
                constexpr int pr = decltype(Pc)::value;
                sfor<0, TS>([&](auto Xc) {
                    constexpr int dx = decltype(Xc)::value, c = ic - dx;
                    if constexpr (c >= 0 && c < S_CW) {
                        const f16x8 &a = pr == 0 ? al[buf] : ah[buf];
                        const f16x8 &b = pr == 1 ? bl[d & 1][dx] : bh[d & 1][dx];
                        acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc[c], 0, 0, 0);
                    }
                });
            });
        });
    };

    // epilogue of tile t from registers: lane (ml, hl) holds pixel m = ml of each of its columns; after the
    // permlane32 regroup, channels 32 nt + 8 (2 s + hl) + e (e < 8) in acc[c][8 s + e]
    const esr_conv_out &o = p.o;
    const int HP = p.H + 2;
    auto epilogue = [&](int t, int ncw) {
        const int x0 = (t % p.tiles_x) * TWC, r0 = (t / p.tiles_x) * CT;
        const int R = r0 + 1 + ml;
        const int b = R / HP, y = R - b * HP - 1;
        const bool vrow = R < rows_tot && y >= 0 && y < p.H;
        bool ok = true;
#pragma unroll 1
        for (int c = 0; c < ncw; ++c) {  // a runtime loop: one column's registers live at a time
            f32x16 a;
            switch (c) {
            case 0: a = acc[0]; break;
            case 1: a = acc[1]; break;
            case 2: a = acc[2]; break;
            default: a = acc[3]; break;
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[8 * s2 + k]),
                                                                    __float_as_uint(a[8 * s2 + 4 + k]), false, false);
                    a[8 * s2 + k] = __uint_as_float(r[0]);
                    a[8 * s2 + 4 + k] = __uint_as_float(r[1]);
                }
            const int x = x0 + S_CW * cw + c;
            const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
            const long long opix = ((long long)b * (o.out_h + 2) + oy + 1) * (long long)(o.out_w + 2) + ox + 1;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int ch = 32 * nt + 8 * (2 * s2 + hl);
                if (!vrow || ch >= p.cout || (DBG & 4)) continue;
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
        if (!ok && p.overflow) atomicOr(p.overflow, 1);
    };

    if (is_loader) {
        if (nunits > 0) dma(0);
        wait_vm0();
    }
    __builtin_amdgcn_s_barrier();
    int cur_tile = x3s_tile(blockIdx.x, gridDim.x, ntiles, 0);
    int j = 0, k = 0;
    for (int u = 0; u < nunits; ++u) {
        if (is_loader) {
            if (u + 1 < nunits && !(DBG & 1)) dma(u + 1);
            wait_vm0();
        } else {
            const int ncw = min(S_CW, max(0, min(TWC, p.W - (cur_tile % p.tiles_x) * TWC) - S_CW * cw));
            if (ncw > 0 && !(DBG & 2)) compute((u & 1) * STAGE);
            if (j == nchunk - 1) {
#ifdef X3S_KEEP_ONLY
#pragma unroll
                for (int c = 0; c < S_CW; ++c) asm volatile("" : "+v"(acc[c]));
#else
                if (ncw > 0) epilogue(cur_tile, ncw);
#endif
                zero_acc();
            }
        }
        if (++j == nchunk) {
            j = 0;
            cur_tile = x3s_tile(blockIdx.x, gridDim.x, ntiles, ++k);
        }
        __builtin_amdgcn_s_barrier();
    }
}

#endif  // ESR_X3_EXPERIMENTS

}  // namespace

static int n_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0, v = 0;
        n = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
    }
    return n;
}

#ifdef ESR_X3_EXPERIMENTS
int x3s_launch(const X3cParams &p0, int taps_side, hipStream_t stream, int dbg) {
    X3cParams p = p0;
    p.tiles_x = (p.W + TWC - 1) / TWC;
    p.tiles_y = (p.B * (p.H + 2) - 2 + CT - 1) / CT;
    const int ntiles = p.tiles_x * p.tiles_y;
    const dim3 grid((unsigned)min(ntiles, n_cus()));
    const bool n64 = p.cout > 32;
#ifdef ESR_X3_EXPERIMENTS
    if (taps_side == 3 && dbg) {
#define XD(f) if (n64) hipLaunchKernelGGL((conv_x3s_kernel<2, 3, f>), grid, dim3(X3sShape<2>::NTHR), 0, stream, p); \
              else hipLaunchKernelGGL((conv_x3s_kernel<1, 3, f>), grid, dim3(X3sShape<1>::NTHR), 0, stream, p)
        switch (dbg) {
        case 1: XD(1); break;
        case 2: XD(2); break;
        case 4: XD(4); break;
        default: XD(1 | 4);
        }
#undef XD
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#else
    (void)dbg;
#endif
    const dim3 b1(X3sShape<1>::NTHR), b2(X3sShape<2>::NTHR);
    if (taps_side == 3) {
        if (n64) hipLaunchKernelGGL((conv_x3s_kernel<2, 3>), grid, b2, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3s_kernel<1, 3>), grid, b1, 0, stream, p);
    } else {
        if (n64) hipLaunchKernelGGL((conv_x3s_kernel<2, 2>), grid, b2, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3s_kernel<1, 2>), grid, b1, 0, stream, p);
    }
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}
#endif

int x3c_launch_hr1(const X3cParams &p0, hipStream_t stream) {
    X3cParams p = p0;
    p.tiles_x = (p.W + TWC - 1) / TWC;
    p.tiles_y = (p.B * (p.H + 2) - 2 + CT - 1) / CT;
    const dim3 grid((unsigned)(p.tiles_x * p.tiles_y)), block(NTHR);
    hipLaunchKernelGGL((conv_x3c_kernel<2, 3, 0, false, CW, false, TWC, 2, true>), grid, block, 0, stream, p);
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

namespace {

// HR_conv1's output from the fused HR_conv0 launch's partial products: out[b][o][y][x] = scale_inv · Σ_t
// Y[b][y + ty][x + tx][3t + o] + bias[o] over the padded Y grid (zero halo).  A block stages the Y records of its
// 18 × 34 padded window in LDS (27 floats each at an odd pitch: conflict-free column reads; 66 KB, two blocks per CU;
// all of a thread's 16-B loads in flight before one barrier), each thread sums two pixels (rows ty and ty + 8).
constexpr int HS_TY = 16, HS_TX = 32, HS_WY = HS_TY + 2, HS_WX = HS_TX + 2, HS_P = 27;
constexpr int HS_Q = HS_WY * HS_WX * 7;                 // 16-B pieces of the window (7 per 28-float record prefix)
constexpr int HS_QT = (HS_Q + 255) / 256;               // per thread

__global__ __launch_bounds__(256) void hr1_sum_kernel(const float *y, int H, int W, const float *bias, float sinv,
                                                      float *out) {
    __shared__ float s[HS_WY * HS_WX * HS_P];
    const int b = blockIdx.z, x0 = blockIdx.x * HS_TX, y0 = blockIdx.y * HS_TY;
    const long long rowp = W + 2;
    const float *yb = y + (long long)b * (H + 2) * rowp * 32;
    f32x4 v[HS_QT];
#pragma unroll
    for (int k = 0; k < HS_QT; ++k) {
        const int i = threadIdx.x + 256 * k;
        const int q = i % 7, rc = i / 7, c = rc % HS_WX, r = rc / HS_WX;
        const int py = y0 + r, px = x0 + c;
        v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (i < HS_Q && py < H + 2 && px < W + 2)
            v[k] = *reinterpret_cast<const f32x4 *>(yb + ((long long)py * rowp + px) * 32 + 4 * q);
    }
#pragma unroll
    for (int k = 0; k < HS_QT; ++k) {
        const int i = threadIdx.x + 256 * k;
        if (i >= HS_Q) break;
        const int q = i % 7, rc = i / 7;
        float *d = s + rc * HS_P + 4 * q;
        d[0] = v[k][0];
        d[1] = v[k][1];
        d[2] = v[k][2];
        if (q < 6) d[3] = v[k][3];
    }
    __syncthreads();
    const int tx = threadIdx.x % HS_TX, xx = x0 + tx;
    if (xx >= W) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int ty = threadIdx.x / HS_TX + 8 * h, yy = y0 + ty;
        if (yy >= H) break;
        float a[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const float *rec = s + ((ty + t / 3) * HS_WX + tx + t % 3) * HS_P + 3 * t;
#pragma unroll
            for (int o = 0; o < 3; ++o) a[o] += rec[o];
        }
#pragma unroll
        for (int o = 0; o < 3; ++o) out[(((long long)b * 3 + o) * H + yy) * W + xx] = a[o] * sinv + bias[o];
    }
}

}  // namespace

int hr1_sum_launch(const float *y, int B, int H, int W, const float *bias, float sinv, float *out, hipStream_t st) {
    const dim3 grid((unsigned)((W + HS_TX - 1) / HS_TX), (unsigned)((H + HS_TY - 1) / HS_TY), (unsigned)B);
    hipLaunchKernelGGL(hr1_sum_kernel, grid, dim3(256), 0, st, y, H, W, bias, sinv, out);
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

int x3c_launch(const X3cParams &p0, int taps_side, hipStream_t stream, int dbg) {
    X3cParams p = p0;
    p.tiles_x = (p.W + TWC - 1) / TWC;
    p.tiles_y = (p.B * (p.H + 2) - 2 + CT - 1) / CT;
    const dim3 grid((unsigned)(p.tiles_x * p.tiles_y)), block(NTHR);
    const bool n64 = p.cout > 32;
#ifdef ESR_X3_EXPERIMENTS  // A/B forms (bitwise identical): the ablation library only
    if (dbg == 32) {  // 8 waves of 2 columns (N = 32 only: the per-wave epilogue areas of N = 64 do not fit)
        const dim3 block8(64 * (TWC / 2));
        if (taps_side == 3 && !n64) hipLaunchKernelGGL((conv_x3c_kernel<1, 3, 0, false, 2>), grid, block8, 0, stream, p);
        else if (!n64) hipLaunchKernelGGL((conv_x3c_kernel<1, 2, 0, false, 2>), grid, block8, 0, stream, p);
        else return x3c_launch(p0, taps_side, stream, 0);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if (dbg == 64) {  // N = 32: weights copied to registers per chunk, the next chunk's weights DMA'd under compute
        if (n64) return x3c_launch(p0, taps_side, stream, 0);
        if (taps_side == 3) hipLaunchKernelGGL((conv_x3c_kernel<1, 3, 0, false, 4, true>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3c_kernel<1, 2, 0, false, 4, true>), grid, block, 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#endif
#ifdef ESR_X3_EXPERIMENTS
    if (dbg >= 256 && dbg < 300 && !n64 && taps_side == 3) {  // 12-column N = 32 kernel ablations: DBG = dbg >> 8
        p.tiles_x = (p.W + 11) / 12;
        const dim3 grid12((unsigned)(p.tiles_x * p.tiles_y));
#define X12(D) hipLaunchKernelGGL((conv_x3c_kernel<1, 3, D, false, 3, false, 12, 3>), grid12, block, 0, stream, p)
        switch (dbg >> 8) {
        case 5: X12(5); break;
        case 13: X12(13); break;
        case 21: X12(21); break;
        case 29: X12(29); break;
        default: X12(0);
        }
#undef X12
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#endif
#ifdef ESR_X3_EXPERIMENTS
    if (dbg == 303 && !n64 && taps_side == 3) {  // the 8-channel double-buffered form (conv_x3d_kernel)
        p.tiles_x = (p.W + 11) / 12;
        const dim3 grid12((unsigned)(p.tiles_x * p.tiles_y));
        hipLaunchKernelGGL(conv_x3d_kernel, grid12, block, 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if (dbg == 302 && !n64 && taps_side == 3) {  // the production 12-column N = 32 kernel with stamps (DBG 32)
        p.tiles_x = (p.W + 11) / 12;
        const dim3 grid12((unsigned)(p.tiles_x * p.tiles_y));
        p.y1 = static_cast<float *>(g_x3c_stamps);
        hipLaunchKernelGGL((conv_x3c_kernel<1, 3, 32, false, 3, false, 12, 3>), grid12, block, 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if ((dbg == 300 || dbg == 301) && !n64 && taps_side == 3) {  // N = 32 in wider tiles at two workgroups per CU:
        // 18 columns (six 3-column waves, 62.5 KB LDS) / 24 columns (eight, 75.8 KB): fewer staged bytes per output
        // pixel (108 / 98 B vs 127 B at 12 columns)
        const int tw = dbg == 300 ? 18 : 24;
        p.tiles_x = (p.W + tw - 1) / tw;
        const dim3 gridw((unsigned)(p.tiles_x * p.tiles_y));
        if (dbg == 300)
            hipLaunchKernelGGL((conv_x3c_kernel<1, 3, 0, false, 3, false, 18, 2>), gridw, dim3(64 * 6), 0, stream, p);
        else
            hipLaunchKernelGGL((conv_x3c_kernel<1, 3, 0, false, 3, false, 24, 2>), gridw, dim3(64 * 8), 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#endif
    if (dbg == 129 && n64) {  // N = 64 in 12-column tiles of four 3-column waves, two workgroups per CU (67.6 KB LDS)
        p.tiles_x = (p.W + 11) / 12;
        const dim3 grid12((unsigned)(p.tiles_x * p.tiles_y));
        if (taps_side == 3) hipLaunchKernelGGL((conv_x3c_kernel<2, 3, 0, false, 3, false, 12, 2>), grid12, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3c_kernel<2, 2, 0, false, 3, false, 12, 2>), grid12, block, 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if (dbg == 128) {  // N = 32: 12-column tiles of four 3-column waves, three workgroups per CU (48 KB LDS, <= 168 VGPRs)
        if (n64) return x3c_launch(p0, taps_side, stream, 0);
        p.tiles_x = (p.W + 11) / 12;
        const dim3 grid12((unsigned)(p.tiles_x * p.tiles_y));
        if (taps_side == 3) hipLaunchKernelGGL((conv_x3c_kernel<1, 3, 0, false, 3, false, 12, 3>), grid12, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3c_kernel<1, 2, 0, false, 3, false, 12, 3>), grid12, block, 0, stream, p);
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#ifdef ESR_X3_EXPERIMENTS
    if (dbg == 16) {  // register-B form
        if (taps_side == 3) {
            if (n64) hipLaunchKernelGGL((conv_x3c_kernel<2, 3, 0, true>), grid, block, 0, stream, p);
            else hipLaunchKernelGGL((conv_x3c_kernel<1, 3, 0, true>), grid, block, 0, stream, p);
        } else {
            if (n64) hipLaunchKernelGGL((conv_x3c_kernel<2, 2, 0, true>), grid, block, 0, stream, p);
            else hipLaunchKernelGGL((conv_x3c_kernel<1, 2, 0, true>), grid, block, 0, stream, p);
        }
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
    if (taps_side == 3 && dbg) {
#define XD(f) if (n64) hipLaunchKernelGGL((conv_x3c_kernel<2, 3, f>), grid, block, 0, stream, p); \
              else hipLaunchKernelGGL((conv_x3c_kernel<1, 3, f>), grid, block, 0, stream, p)
        switch (dbg) {
        case 1: XD(1); break;
        case 2: XD(2); break;
        case 4: XD(4); break;
        default: XD(1 | 4);
        }
#undef XD
        return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
    }
#else
    (void)dbg;
#endif
    if (taps_side == 3) {
        if (n64) hipLaunchKernelGGL((conv_x3c_kernel<2, 3>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3c_kernel<1, 3>), grid, block, 0, stream, p);
    } else {
        if (n64) hipLaunchKernelGGL((conv_x3c_kernel<2, 2>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3c_kernel<1, 2>), grid, block, 0, stream, p);
    }
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

#ifdef ESR_X3_EXPERIMENTS
// variant 87's stamp buffer (X3C_NS u64 per workgroup of the launch; NULL: stamps not stored)
extern "C" int esr_x3c_set_stamps(void *buf) {
    g_x3c_stamps = buf;
    return 0;
}
#endif
