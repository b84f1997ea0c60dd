// esr_cem.hip — Consistency Enforcing Module (CEM) stencils and model-input preparation for gfx950.
//
// The CEM step (CEMnet.py:184-190) is  out = Up(Inv(LR)) + gen - Up(Inv(Down(gen)))  with three fixed depthwise
// filters.  By linearity it equals  gen + Up(Inv(LR - Down(gen))),  which we evaluate as three HBM-bound stencil
// passes with exact reference indexing:
//   esr_cem_down   : r = LR - Down(gen)            polyphase: only the sf-strided phase of the ×sf grid is computed
//   esr_cem_inv    : q = Inv(r)                    replicate-padded depthwise xcorr at LR resolution
//   esr_cem_up_add : out = crop(gen + Up(q))       zero-stuffed ×sf grid never materialised; only taps that land on
//                                                 a stuffed sample are visited
// Replicate padding is realised as index clamping (ReplicationPad2d, CEMnet.py:63-64,150,158).
#include <hip/hip_runtime.h>
#include "esr_amd.h"
#include "esr_knobs.h"

namespace {

constexpr int NT = 256;
constexpr int MAXK = 64;  // largest supported filter side

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__global__ __launch_bounds__(NT) void cem_down_kernel(const float *__restrict__ gen, const float *__restrict__ lr,
                                                      float *__restrict__ r, int B, int H, int W, int sf, int ph,
                                                      const float *__restrict__ wd, int kd, int negate) {
    __shared__ float sw[MAXK * MAXK];
    for (int i = threadIdx.x; i < kd * kd; i += NT) sw[i] = wd[i];
    __syncthreads();
    const long long total = (long long)B * 3 * H * W;
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= total) return;
    const int j = idx % W;
    const int i = (idx / W) % H;
    const long long plane = idx / ((long long)H * W);  // b*3 + c
    const int HH = sf * H, WW = sf * W;
    const float *g = gen + plane * HH * WW;
    const int pd = kd / 2;
    const int ry = sf * i + ph - pd, rx = sf * j + ph - pd;
    float acc = 0.f;
    for (int u = 0; u < kd; ++u) {
        const float *grow = g + (long long)clampi(ry + u, 0, HH - 1) * WW;
        const float *wrow = sw + u * kd;
        for (int v = 0; v < kd; ++v) acc += wrow[v] * grow[clampi(rx + v, 0, WW - 1)];
    }
    float out = (lr ? lr[idx] : 0.f) - acc;
    r[idx] = negate ? -out : out;
}

__global__ __launch_bounds__(NT) void cem_inv_kernel(const float *__restrict__ rin, float *__restrict__ q, int B,
                                                     int H, int W, const float *__restrict__ wi, int ki) {
    __shared__ float sw[MAXK * MAXK];
    for (int i = threadIdx.x; i < ki * ki; i += NT) sw[i] = wi[i];
    __syncthreads();
    const long long total = (long long)B * 3 * H * W;
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= total) return;
    const int j = idx % W;
    const int i = (idx / W) % H;
    const long long plane = idx / ((long long)H * W);
    const float *src = rin + plane * H * W;
    const int pd = ki / 2;
    float acc = 0.f;
    for (int u = 0; u < ki; ++u) {
        const float *row = src + (long long)clampi(i + u - pd, 0, H - 1) * W;
        const float *wrow = sw + u * ki;
        for (int v = 0; v < ki; ++v) acc += wrow[v] * row[clampi(j + v - pd, 0, W - 1)];
    }
    q[idx] = acc;
}

__global__ __launch_bounds__(NT) void cem_up_add_kernel(const float *__restrict__ q, const float *__restrict__ gen,
                                                        float *__restrict__ out, int B, int H, int W, int sf, int ph,
                                                        const float *__restrict__ wu, int kd, int M) {
    __shared__ float sw[MAXK * MAXK];
    for (int i = threadIdx.x; i < kd * kd; i += NT) sw[i] = wu[i];
    __syncthreads();
    const int HH = sf * H, WW = sf * W;
    const int OH = HH - 2 * M, OW = WW - 2 * M;
    const long long total = (long long)B * 3 * OH * OW;
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= total) return;
    const int X = idx % OW;
    const int Y = (idx / OW) % OH;
    const long long plane = idx / ((long long)OH * OW);
    const float *qp = q + plane * H * W;
    const int pd = kd / 2;
    float acc = 0.f;
    for (int u = 0; u < kd; ++u) {
        const int py = clampi(Y + M + u - pd, 0, HH - 1) - ph;  // position in the stuffed grid, relative to phase
        if (py < 0 || py % sf) continue;
        const float *qrow = qp + (long long)(py / sf) * W;
        const float *wrow = sw + u * kd;
        for (int v = 0; v < kd; ++v) {
            const int px = clampi(X + M + v - pd, 0, WW - 1) - ph;
            if (px < 0 || px % sf) continue;
            acc += wrow[v] * qrow[px / sf];
        }
    }
    out[idx] = gen[(plane * HH + Y + M) * WW + X + M] + acc;
}

// ---- tiled forms (the launchers use these; the direct kernels above remain for the general stride phase) ----------
// Down: a 16×16 block of LR outputs of one plane stages its replicate-clamped HR window ((15·sf+kd)² values) in LDS,
// de-interleaved by column phase (x mod sf) so that lanes reading columns sf·j + v hit consecutive words.
template <int sf>
__global__ __launch_bounds__(256) void cem_down_tiled(const float *__restrict__ gen, const float *__restrict__ lr,
                                                      float *__restrict__ r, int H, int W, int ph,
                                                      const float *__restrict__ wd, int kd, int negate) {
    extern __shared__ float smem[];
    const int WH = 15 * sf + kd;              // window rows = cols
    const int P = (WH + sf - 1) / sf + 1;     // de-interleaved row pitch (+1: bank spread)
    float *sw = smem;                         // kd*kd weights
    float *s = smem + ((kd * kd + 3) & ~3);   // [sf][WH][P]
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int j0 = blockIdx.x * 16, i0 = blockIdx.y * 16;
    const long long plane = blockIdx.z;
    const int HH = sf * H, WW = sf * W, pd = kd / 2;
    const float *g = gen + plane * HH * WW;
    for (int k = threadIdx.x; k < kd * kd; k += 256) sw[k] = wd[k];
    const int Y0 = sf * i0 + ph - pd, X0 = sf * j0 + ph - pd;
    // 64 lanes along a window row (coalesced), 4 rows per pass, 8 passes' loads in flight before their LDS stores
    // (one load at a time made the staging latency-bound); WH <= 128 (kd <= 64), no integer division
    const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
    for (int yb = ly; yb < WH; yb += 32) {
        float v[8][2];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float *grow = g + (long long)clampi(Y0 + yb + 4 * e, 0, HH - 1) * WW;
#pragma unroll
            for (int h = 0; h < 2; ++h) v[e][h] = grow[clampi(X0 + lx + 64 * h, 0, WW - 1)];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int y = yb + 4 * e, x = lx + 64 * h;
                if (y < WH && x < WH) s[((x & (sf - 1)) * WH + y) * P + x / sf] = v[e][h];
            }
    }
    __syncthreads();
    const int i = i0 + ty, j = j0 + tx;
    if (i >= H || j >= W) return;
    float acc = 0.f;
    for (int u = 0; u < kd; ++u) {
        const float *wrow = sw + u * kd;
        const float *srow = s + (sf * ty + u) * P + tx;
        for (int v0 = 0; v0 < kd; v0 += sf) {  // v = v0 + ph_: phase ph_, de-interleaved index v0/sf
#pragma unroll
            for (int ph_ = 0; ph_ < sf; ++ph_)
                if (v0 + ph_ < kd) acc += wrow[v0 + ph_] * srow[ph_ * WH * P + v0 / sf];
        }
    }
    const long long idx = (plane * H + i) * W + j;
    const float out = (lr ? lr[idx] : 0.f) - acc;
    r[idx] = negate ? -out : out;
}

// Down, register-window form (sf = 4): a 32×16 block of LR outputs of one plane stages its replicate-clamped HR window
// (77 × 141 values for kd = 17) in LDS de-interleaved by column phase x mod 4, rows padded to P ≡ 8 (mod 16) words.
// Thread (tx, ty) owns the 4 consecutive outputs j0 + 4 tx + e of row i0 + ty: for every tap row u it reads the 8
// values [4 tx, 4 tx + 8) of each phase row with two ds_read_b128 (conflict-free: 8 lanes cover 128 B of one row, the
// next row group starts 32 banks later), i.e. 8 LDS reads per tap row for 4·kd FMAs, and the weights are broadcast
// LDS reads.  Per output the taps are summed u-major, v ascending — the order of cem_down_tiled: bitwise equal.
constexpr int DW_TX = 8, DW_TY = 16;  // 32 × 16 LR outputs, 128 threads
// The window is staged from the 16-B-aligned column Xa = X0 & ~3 (O = X0 - Xa, a template parameter) with 16-B loads
// (per-element clamped loads only where a 16-B group crosses the image border), all of a thread's loads in flight
// before its LDS stores.
template <int KD, int O>
__global__ __launch_bounds__(128) void cem_down_win4(const float *__restrict__ gen, const float *__restrict__ lr,
                                                     float *__restrict__ r, int H, int W, int ph,
                                                     const float *__restrict__ wd, int negate) {
    constexpr int sf = 4, kd = KD;
    static_assert(KD + O <= 20, "8-value windows cover taps v + O < 20");
    constexpr int WR = (DW_TY - 1) * sf + kd;             // window rows
    constexpr int WC4 = ((4 * DW_TX - 1) * sf + kd + O + 3) / 4;  // 16-B column groups from Xa
    constexpr int P = ((WC4 + 7) & ~15) + 8;              // >= WC4, ≡ 8 (mod 16) words
    constexpr int NL = (WR * WC4 + 127) / 128;            // 16-B loads per thread
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __shared__ float sw[KD * KD];  // the taps, read from LDS (broadcast), not as scalar loads: see cem_inv_tiled
    for (int k = threadIdx.x; k < KD * KD; k += 128) sw[k] = wd[k];
    const int j0 = blockIdx.x * 4 * DW_TX, i0 = blockIdx.y * DW_TY;
    const long long plane = blockIdx.z;
    const int HH = sf * H, WW = sf * W, pd = kd / 2;
    const float *g = gen + plane * HH * WW;
    const int Y0 = sf * i0 + ph - pd, Xa = sf * j0 + ph - pd - O;
    float4 v[NL];
#pragma unroll
    for (int n = 0; n < NL; ++n) {
        const int k = threadIdx.x + 128 * n, y = k / WC4, c = k - y * WC4;
        if (y < WR) {
            const float *grow = g + (long long)clampi(Y0 + y, 0, HH - 1) * WW;
            const int x = Xa + 4 * c;
            if (x >= 0 && x + 3 < WW) {
                v[n] = *reinterpret_cast<const float4 *>(grow + x);
            } else {
                v[n].x = grow[clampi(x, 0, WW - 1)];
                v[n].y = grow[clampi(x + 1, 0, WW - 1)];
                v[n].z = grow[clampi(x + 2, 0, WW - 1)];
                v[n].w = grow[clampi(x + 3, 0, WW - 1)];
            }
        }
    }
#pragma unroll
    for (int n = 0; n < NL; ++n) {
        const int k = threadIdx.x + 128 * n, y = k / WC4, c = k - y * WC4;
        if (y < WR) {
            smem[(0 * WR + y) * P + c] = v[n].x;
            smem[(1 * WR + y) * P + c] = v[n].y;
            smem[(2 * WR + y) * P + c] = v[n].z;
            smem[(3 * WR + y) * P + c] = v[n].w;
        }
    }
    __syncthreads();
    const int tx = threadIdx.x % DW_TX, ty = threadIdx.x / DW_TX;
    const int i = i0 + ty, j = j0 + 4 * tx;
    if (i >= H || j >= W) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int u = 0; u < kd; ++u) {
        float win[4][8];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 *src = reinterpret_cast<const float4 *>(smem + (q * WR + sf * ty + u) * P + 4 * tx);
            const float4 a = src[0], b = src[1];
            win[q][0] = a.x; win[q][1] = a.y; win[q][2] = a.z; win[q][3] = a.w;
            win[q][4] = b.x; win[q][5] = b.y; win[q][6] = b.z; win[q][7] = b.w;
        }
        const float *wr = sw + u * kd;  // wave-uniform row, broadcast LDS reads
#pragma unroll
        for (int vv = 0; vv < kd; ++vv) {
            const float w = wr[vv];
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] += w * win[(vv + O) & 3][e + ((vv + O) >> 2)];
        }
    }
    const long long idx = (plane * H + i) * W + j;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        if (j + e >= W) break;
        const float out = (lr ? lr[idx + e] : 0.f) - acc[e];
        r[idx + e] = negate ? -out : out;
    }
}

// Up + back-projection + crop, for stride phases whose clamped border rows/columns are not stuffed rows
// (0 < ph < sf-1: replicate padding of the zero-stuffed grid then reads zeros): only the ≈(kd/sf)² taps that land on
// stuffed samples are visited, with no modulo in the tap loops.
template <int sf>
__global__ __launch_bounds__(256) void cem_up_add_phase(const float *__restrict__ q, const float *__restrict__ gen,
                                                        float *__restrict__ out, int H, int W, int ph,
                                                        const float *__restrict__ wu, int kd, int M) {
    __shared__ float sw[MAXK * MAXK];
    for (int k = threadIdx.x; k < kd * kd; k += 256) sw[k] = wu[k];
    __syncthreads();
    const int HH = sf * H, WW = sf * W, OH = HH - 2 * M, OW = WW - 2 * M;
    const int X = blockIdx.x * 64 + (threadIdx.x & 63), Y = blockIdx.y * 4 + (threadIdx.x >> 6);
    const long long plane = blockIdx.z;
    if (X >= OW || Y >= OH) return;
    const int pd = kd / 2, Yp = Y + M, Xp = X + M;
    // first tap on a stuffed row/column: (Yp + u - pd - ph) ≡ 0 (mod sf); the +sf·kd keeps the operand positive
    const int u0 = (pd + ph - Yp + sf * (Yp + kd)) % sf, v0 = (pd + ph - Xp + sf * (Xp + kd)) % sf;
    const float *qp = q + plane * H * W;
    float acc = 0.f;
    for (int u = u0; u < kd; u += sf) {
        const int py = Yp + u - pd;
        if (py < 0 || py >= HH) continue;
        const float *qrow = qp + (long long)((py - ph) / sf) * W;
        const float *wrow = sw + u * kd;
        for (int v = v0; v < kd; v += sf) {
            const int px = Xp + v - pd;
            if (px < 0 || px >= WW) continue;
            acc += wrow[v] * qrow[(px - ph) / sf];
        }
    }
    out[(plane * OH + Y) * OW + X] = gen[(plane * HH + Yp) * WW + Xp] + acc;
}

// Inverse filter, tiled: a 64×16 block of outputs of one plane stages its replicate-clamped (16+ki-1)×(64+ki-1) input
// window in LDS once (the direct kernel re-read every input ki² times through L1/L2, with a clamp per tap); each thread
// owns 4 consecutive outputs of a row and slides a 4-wide register window along each tap row, so one LDS read feeds
// 4 FMAs.  Accumulation order per output (u-major, v-minor) is the direct kernel's: results are bitwise equal.
__global__ __launch_bounds__(256) void cem_inv_tiled(const float *__restrict__ rin, float *__restrict__ q, int H, int W,
                                                     const float *__restrict__ wi, int ki) {
    extern __shared__ float smem[];
    const int WP = 64 + ki - 1, WR = 16 + ki - 1;
    float *s = smem;                           // [WR][WP]
    // The taps are read from LDS (broadcast), not as wave-uniform scalar loads: with SGPR operands the compiler
    // emitted packed FMAs (v_pk_fma_f32 s[n:n+1]) whose SGPRs the loop's next s_load overwrote, and under concurrent
    // kernels on the CU the upper lanes of a wave then read the next row's taps (tools/race_probe.py: outputs of two
    // identical processes in lockstep differed in lanes 48-63 of one packed result).
    float *sw = smem + WR * WP;
    for (int k = threadIdx.x; k < ki * ki; k += 256) sw[k] = wi[k];
    const int j0 = blockIdx.x * 64, i0 = blockIdx.y * 16;
    const long long plane = blockIdx.z;
    const float *src = rin + plane * H * W;
    const int pd = ki / 2;
    const int lx = threadIdx.x & 63, ly = threadIdx.x >> 6;
    for (int yb = ly; yb < WR; yb += 32) {  // 8 passes' loads in flight before their stores (WP <= 128)
        float v[8][2];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float *row = src + (long long)clampi(i0 + yb + 4 * e - pd, 0, H - 1) * W;
#pragma unroll
            for (int h = 0; h < 2; ++h) v[e][h] = row[clampi(j0 + lx + 64 * h - pd, 0, W - 1)];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int y = yb + 4 * e, x = lx + 64 * h;
                if (y < WR && x < WP) s[y * WP + x] = v[e][h];
            }
    }
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    for (int u = 0; u < ki; ++u) {
        const float *sr = s + (ty + u) * WP + 4 * tx;
        const float *wr = sw + u * ki;  // broadcast LDS reads
        float r0 = sr[0], r1 = sr[1], r2 = sr[2];
#pragma unroll 4
        for (int v = 0; v < ki; ++v) {
            const float r3 = sr[v + 3], w = wr[v];
            a0 += w * r0;
            a1 += w * r1;
            a2 += w * r2;
            a3 += w * r3;
            r0 = r1;
            r1 = r2;
            r2 = r3;
        }
    }
    const int i = i0 + ty, j = j0 + 4 * tx;
    if (i >= H) return;
    float *qo = q + (plane * H + i) * W;
    if (j < W) qo[j] = a0;
    if (j + 1 < W) qo[j + 1] = a1;
    if (j + 2 < W) qo[j + 2] = a2;
    if (j + 3 < W) qo[j + 3] = a3;
}

// Up + back-projection + crop, tiled (interior stride phases, as cem_up_add_phase): a 64×16 block of cropped HR outputs
// of one plane stages the q window its taps can reach in LDS, zero outside [0,H)×[0,W) — exactly the taps the phase
// kernel skips (for 0 < ph < sf-1 a tap outside the HR grid, or on a clamped border row, is not a stuffed sample) — so
// the tap loops have no bounds tests: each output visits the (kd/sf)² taps of its own sub-pixel phase, u0 + sf·a,
// v0 + sf·b, reading q[r + a][c + b].  Same taps in the same order as cem_up_add_phase: bitwise equal.
template <int sf, int RPT>
__global__ __launch_bounds__(256) void cem_up_add_tiled(const float *__restrict__ q, const float *__restrict__ gen,
                                                        float *__restrict__ out, int H, int W, int ph,
                                                        const float *__restrict__ wu, int kd, int M) {
    extern __shared__ float smem[];
    float *sw = smem;
    const int QC = (63 + kd - 1) / sf + 3, QR = (16 * RPT - 1 + kd - 1) / sf + 3;
    float *sq = smem + ((kd * kd + 3) & ~3);  // [QR][QC]
    const int HH = sf * H, WW = sf * W, OH = HH - 2 * M, OW = WW - 2 * M;
    const int X0 = blockIdx.x * 64, Y0 = blockIdx.y * 16 * RPT;
    const long long plane = blockIdx.z;
    const int pd = kd / 2;
    // q row of the first tap of the block's first output row, minus one (floor division of a possibly negative value)
    const int qr0 = (Y0 + M - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - 1;
    const int qc0 = (X0 + M - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - 1;
    // thread (tx, ty): the 4 consecutive outputs X0 + 4 tx + e (e < 4) of rows Y0 + ty + 16 k (k < RPT); one 16-B gen
    // load and one 16-B store per 4 outputs when rows are 16-B aligned (WW, OW, M multiples of 4), else per element.
    // The gen loads are issued before the q window is staged, so their latency hides behind the staging and taps.
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 column groups x 16 rows
    const int Xb = X0 + 4 * tx;
    const bool vec = ((WW | OW | M) & 3) == 0 && Xb + 4 <= OW;
    float4 gv[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int Y = Y0 + ty + 16 * k;
        const float *g = gen + (plane * HH + min(Y, OH - 1) + M) * WW + min(Xb, OW - 1) + M;
        if (vec) {
            gv[k] = *reinterpret_cast<const float4 *>(g);
        } else {
            gv[k].x = g[0];
            gv[k].y = Xb + 1 < OW ? g[1] : 0.f;
            gv[k].z = Xb + 2 < OW ? g[2] : 0.f;
            gv[k].w = Xb + 3 < OW ? g[3] : 0.f;
        }
    }
    for (int k = threadIdx.x; k < kd * kd; k += 256) sw[k] = wu[k];
    const float *qp = q + plane * H * W;
    for (int k = threadIdx.x; k < QR * QC; k += 256) {
        const int r = k / QC, c = k - r * QC;
        const int qr = qr0 + r, qc = qc0 + c;
        sq[k] = (qr >= 0 && qr < H && qc >= 0 && qc < W) ? qp[(long long)qr * W + qc] : 0.f;
    }
    __syncthreads();
    if (Xb >= OW) return;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int Y = Y0 + ty + 16 * k;
        if (Y >= OH) return;
        const int Yp = Y + M;
        const int u0 = (pd + ph - Yp + sf * (Yp + kd)) % sf;
        const int rb = (Yp + u0 - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - qr0;
        float acc[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int Xp = Xb + e + M;
            const int v0 = (pd + ph - Xp + sf * (Xp + kd)) % sf;
            const int cb = (Xp + v0 - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - qc0;
            float a_ = 0.f;
            for (int u = u0, a = 0; u < kd; u += sf, ++a) {
                const float *qrow = sq + (rb + a) * QC + cb;
                const float *wrow = sw + u * kd;
                for (int v = v0, b = 0; v < kd; v += sf, ++b) a_ += wrow[v] * qrow[b];
            }
            acc[e] = a_;
        }
        float *o = out + (plane * OH + Y) * OW + Xb;
        if (vec) {
            *reinterpret_cast<float4 *>(o) = make_float4(gv[k].x + acc[0], gv[k].y + acc[1], gv[k].z + acc[2],
                                                         gv[k].w + acc[3]);
        } else {
            const float gg[4] = {gv[k].x, gv[k].y, gv[k].z, gv[k].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (Xb + e < OW) o[e] = gg[e] + acc[e];
        }
    }
}

// Up + back-projection + crop, register-window form (sf 4, 16-B-aligned rows: WW, OW, M multiples of 4; interior
// stride phases as cem_up_add_tiled).  A block covers 4 output rows × 256 columns; wave w owns row Y0 + w, so the tap
// rows u0 + 4a of its sub-pixel row phase — and the weights they use — are wave-uniform (scalar loads).  Lane l owns
// the 4 consecutive outputs Xb = X0 + 4 l + e: their column phases are e, so output e visits taps v = v0_e + 4 b with
// v0_e = (C0 - e) & 3 (C0 = (kd/2 + ph) & 3, a template parameter) and reads q columns cb_0 + [e > C0] + b.  Per tap row
// a lane reads 5 q values (consecutive lanes, consecutive words) for the ≈kd FMAs of its 4 outputs.  Taps per output
// in the order of cem_up_add_tiled (u ascending, then v).
template <int KD, int C0>
__global__ __launch_bounds__(256) void cem_up_add_win4(const float *__restrict__ q, const float *__restrict__ gen,
                                                       float *__restrict__ out, int H, int W, int ph,
                                                       const float *__restrict__ wu, int M) {
    constexpr int sf = 4, kd = KD, pd = KD / 2;
    constexpr int QC = (255 + kd - 1) / sf + 3, QR = (3 + kd - 1) / sf + 3;
    __shared__ float sq[QR * QC];
    __shared__ float sw[KD * KD];  // the taps, read from LDS (broadcast), not as scalar loads: see cem_inv_tiled
    for (int k = threadIdx.x; k < KD * KD; k += 256) sw[k] = wu[k];
    const int HH = sf * H, WW = sf * W, OH = HH - 2 * M, OW = WW - 2 * M;
    const int X0 = blockIdx.x * 256, Y0 = blockIdx.y * 4;
    const long long plane = blockIdx.z;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int qr0 = (Y0 + M - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - 1;
    const int qc0 = (X0 + M - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - 1;
    const int Y = Y0 + wave, Xb = X0 + 4 * lane;
    float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (Y < OH && Xb < OW) gv = *reinterpret_cast<const float4 *>(gen + (plane * HH + Y + M) * WW + Xb + M);
    const float *qp = q + plane * H * W;
    for (int k = threadIdx.x; k < QR * QC; k += 256) {
        const int r = k / QC, c = k - r * QC;
        const int qr = qr0 + r, qc = qc0 + c;
        sq[k] = (qr >= 0 && qr < H && qc >= 0 && qc < W) ? qp[(long long)qr * W + qc] : 0.f;
    }
    __syncthreads();
    if (Y >= OH || Xb >= OW) return;
    const int Yp = Y + M, Xp = Xb + M;
    const int u0 = (pd + ph - Yp + sf * (Yp + kd)) % sf;  // wave-uniform
    const int rb = (Yp + u0 - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - qr0;
    const int cb = (Xp + C0 - pd - ph + sf * (kd + sf)) / sf - (kd + sf) - qc0;  // output 0: v0 = C0
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int u = u0, a = 0; u < kd; u += sf, ++a) {
        const float *qrow = sq + (rb + a) * QC + cb;
        float qv[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) qv[k] = qrow[k];
        const float *wr = sw + u * kd;  // wave-uniform row, broadcast LDS reads
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int v0 = (C0 - e) & 3, off = e > C0 ? 1 : 0;
#pragma unroll
            for (int b = 0; b < 5; ++b)
                if (v0 + sf * b < kd) acc[e] += wr[v0 + sf * b] * qv[off + b];
        }
    }
    *reinterpret_cast<float4 *>(out + (plane * OH + Y) * OW + Xb) =
        make_float4(gv.x + acc[0], gv.y + acc[1], gv.z + acc[2], gv.w + acc[3]);
}

// ---- model-input preparation ----

struct PrepParams {
    const float *x;
    int B, nz, h, w, sf, m, split;
    float ascale;  // split outputs hold v × ascale (a power of two: the x3 forward's activation scale)
    float *lr_nchw;
    float *first;
    int first_cp, first_lr_off;
    float *zlr[4];
    int zlr_cp[4];
    int n_zlr;
    float *zhr[4];
    int zhr_cp[4];
    int n_zhr;
};

// Z_HR (replicate-padded by sf*m) at padded-HR coords (Y, X), channel c.
__device__ __forceinline__ float zhr_at(const PrepParams &p, int b, int c, int Y, int X) {
    const int Hs = p.sf * p.h, Ws = p.sf * p.w;
    const int yy = clampi(Y - p.sf * p.m, 0, Hs - 1), xx = clampi(X - p.sf * p.m, 0, Ws - 1);
    const long long bstride = (long long)(p.nz * p.sf * p.sf + 3) * p.h * p.w;
    return p.x[b * bstride + (long long)c * Hs * Ws + (long long)yy * Ws + xx];
}

// Store channel c of a padded-NHWC pixel record, fp32 or split f16 (hi/lo groups of 8, esr_conv_x3.hip) of v × ascale.
__device__ __forceinline__ void put_ch(float *buf, long long pix, int cp, int c, float v, int split, float ascale) {
    if (!split) {
        buf[pix * cp + c] = v;
        return;
    }
    v *= ascale;
    _Float16 *q = reinterpret_cast<_Float16 *>(reinterpret_cast<unsigned char *>(buf) + (pix * cp + (c & ~7)) * 4);
    const _Float16 hi = (_Float16)v;
    q[c & 7] = hi;
    q[8 + (c & 7)] = (_Float16)(v - (float)hi);
}

__global__ __launch_bounds__(NT) void prep_lr_kernel(PrepParams p) {
    const int H = p.h + 2 * p.m, W = p.w + 2 * p.m;
    const long long total = (long long)p.B * H * W;
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= total) return;
    const int x = idx % W;
    const int y = (idx / W) % H;
    const int b = idx / ((long long)H * W);
    const long long pix = ((long long)b * (H + 2) + y + 1) * (W + 2) + x + 1;
    const long long bstride = (long long)(p.nz * p.sf * p.sf + 3) * p.h * p.w;
    const int sy = clampi(y - p.m, 0, p.h - 1), sx = clampi(x - p.m, 0, p.w - 1);
    const float *lr = p.x + b * bstride + (long long)p.nz * p.sf * p.sf * p.h * p.w;
    for (int c = 0; c < 3; ++c) {
        const float v = lr[(long long)c * p.h * p.w + (long long)sy * p.w + sx];
        if (p.lr_nchw) p.lr_nchw[(((long long)b * 3 + c) * H + y) * W + x] = v;
        if (p.first) put_ch(p.first, pix, p.first_cp, p.first_lr_off + c, v, p.split, p.ascale);
    }
    if (p.nz == 0) return;
    // F.interpolate(scale 1/sf, bilinear, align_corners=False): src = (d+0.5)*sf-0.5
    const float fy = (y + 0.5f) * p.sf - 0.5f, fx = (x + 0.5f) * p.sf - 0.5f;
    const int Hs = p.sf * H, Ws = p.sf * W;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = min(y0 + 1, Hs - 1), x1 = min(x0 + 1, Ws - 1);
    const float ly = fy - y0, lx = fx - x0;
    const float hy0 = 1.f - ly, hx0 = 1.f - lx;
    for (int c = 0; c < p.nz; ++c) {
        const float v = hy0 * (hx0 * zhr_at(p, b, c, y0, x0) + lx * zhr_at(p, b, c, y0, x1)) +
                        ly * (hx0 * zhr_at(p, b, c, y1, x0) + lx * zhr_at(p, b, c, y1, x1));
        if (p.first) put_ch(p.first, pix, p.first_cp, c, v, p.split, p.ascale);
        for (int k = 0; k < p.n_zlr; ++k) put_ch(p.zlr[k], pix, p.zlr_cp[k], c, v, p.split, p.ascale);
    }
}

__global__ __launch_bounds__(NT) void prep_hr_kernel(PrepParams p) {
    const int Hs = p.sf * (p.h + 2 * p.m), Ws = p.sf * (p.w + 2 * p.m);
    const long long total = (long long)p.B * Hs * Ws;
    const long long idx = (long long)blockIdx.x * NT + threadIdx.x;
    if (idx >= total) return;
    const int X = idx % Ws;
    const int Y = (idx / Ws) % Hs;
    const int b = idx / ((long long)Hs * Ws);
    const long long pix = ((long long)b * (Hs + 2) + Y + 1) * (Ws + 2) + X + 1;
    for (int c = 0; c < p.nz; ++c) {
        const float v = zhr_at(p, b, c, Y, X);
        for (int k = 0; k < p.n_zhr; ++k) put_ch(p.zhr[k], pix, p.zhr_cp[k], c, v, p.split, p.ascale);
    }
}

inline unsigned nblocks(long long n) { return (unsigned)((n + NT - 1) / NT); }
inline int launched() { return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH; }

}  // namespace

extern "C" int esr_cem_down(const float *gen, const float *lr, float *r, int32_t B, int32_t H, int32_t W, int32_t sf,
                            int32_t ph, const float *w_down, int32_t kd, int32_t negate, esr_stream_t stream) {
    if (!gen || !r || !w_down || B <= 0 || H <= 0 || W <= 0 || sf <= 0 || kd <= 0 || kd > MAXK || !(kd & 1) ||
        ph < 0 || ph >= sf)
        return ESR_EINVAL;
    const int WH = 15 * sf + kd, P = (WH + sf - 1) / sf + 1;
    const size_t lds = 4 * (((kd * kd + 3) & ~3) + (size_t)sf * WH * P);
    if (sf == 4 && kd == 17 && !g_cem_direct) {
        constexpr int WR = (DW_TY - 1) * 4 + 17;
        const dim3 grid((W + 4 * DW_TX - 1) / (4 * DW_TX), (H + DW_TY - 1) / DW_TY, B * 3);
        const int o = ((ph - kd / 2) % 4 + 4) % 4;  // X0 mod 4 (X0 = 4 j0 + ph - kd/2)
#define DW(O_) { constexpr int WC4 = ((4 * DW_TX - 1) * 4 + 17 + O_ + 3) / 4, PW = ((WC4 + 7) & ~15) + 8; \
            hipLaunchKernelGGL((cem_down_win4<17, O_>), grid, dim3(128), (size_t)4 * 4 * WR * PW, (hipStream_t)stream, \
                               gen, lr, r, H, W, ph, w_down, negate); }
        switch (o) {
        case 0: DW(0) break;
        case 1: DW(1) break;
        case 2: DW(2) break;
        default: DW(3)
        }
#undef DW
    } else if (sf == 4 && lds <= 64 * 1024) {
        hipLaunchKernelGGL(cem_down_tiled<4>, dim3((W + 15) / 16, (H + 15) / 16, B * 3), dim3(256), lds,
                           (hipStream_t)stream, gen, lr, r, H, W, ph, w_down, kd, negate);
    } else {
        hipLaunchKernelGGL(cem_down_kernel, dim3(nblocks((long long)B * 3 * H * W)), dim3(NT), 0, (hipStream_t)stream,
                           gen, lr, r, B, H, W, sf, ph, w_down, kd, negate);
    }
    return launched();
}

extern "C" int esr_cem_inv(const float *r, float *q, int32_t B, int32_t H, int32_t W, const float *w_inv, int32_t ki,
                           esr_stream_t stream) {
    if (!r || !q || !w_inv || B <= 0 || H <= 0 || W <= 0 || ki <= 0 || ki > MAXK || !(ki & 1)) return ESR_EINVAL;
    const size_t lds = 4 * ((size_t)(16 + ki - 1) * (64 + ki - 1) + (size_t)ki * ki);
    if (lds <= 64 * 1024 && !g_cem_direct) {
        hipLaunchKernelGGL(cem_inv_tiled, dim3((W + 63) / 64, (H + 15) / 16, B * 3), dim3(256), lds,
                           (hipStream_t)stream, r, q, H, W, w_inv, ki);
    } else {
        hipLaunchKernelGGL(cem_inv_kernel, dim3(nblocks((long long)B * 3 * H * W)), dim3(NT), 0, (hipStream_t)stream,
                           r, q, B, H, W, w_inv, ki);
    }
    return launched();
}

extern "C" int esr_cem_up_add(const float *q, const float *gen, float *out, int32_t B, int32_t H, int32_t W,
                              int32_t sf, int32_t ph, const float *w_up, int32_t kd, int32_t M, esr_stream_t stream) {
    if (!q || !gen || !out || !w_up || B <= 0 || H <= 0 || W <= 0 || sf <= 0 || kd <= 0 || kd > MAXK || !(kd & 1) ||
        ph < 0 || ph >= sf || M < 0 || 2 * M >= sf * H || 2 * M >= sf * W)
        return ESR_EINVAL;
    if (sf == 4 && ph > 0 && ph < sf - 1) {
        constexpr int RPT = 1;  // rows per thread: 64 x 16 outputs per block (64 x 64 measured slower)
        const int QC = (63 + kd - 1) / sf + 3, QR = (16 * RPT - 1 + kd - 1) / sf + 3;
        const size_t lds = 4 * (((kd * kd + 3) & ~3) + (size_t)QR * QC);
        const int c0 = (kd / 2 + ph) & 3;
        if (!g_cem_direct && kd == 17 && (((sf * W) | (sf * W - 2 * M) | M) & 3) == 0) {
            const dim3 grid((sf * W - 2 * M + 255) / 256, (sf * H - 2 * M + 3) / 4, B * 3);
#define UW(C) hipLaunchKernelGGL((cem_up_add_win4<17, C>), grid, dim3(256), 0, (hipStream_t)stream, q, gen, out, H, W, \
                                 ph, w_up, M)
            switch (c0) {
            case 0: UW(0); break;
            case 1: UW(1); break;
            case 2: UW(2); break;
            default: UW(3);
            }
#undef UW
        } else if (g_cem_direct)
            hipLaunchKernelGGL(cem_up_add_phase<4>, dim3((sf * W - 2 * M + 63) / 64, (sf * H - 2 * M + 3) / 4, B * 3),
                               dim3(256), 0, (hipStream_t)stream, q, gen, out, H, W, ph, w_up, kd, M);
        else
            hipLaunchKernelGGL((cem_up_add_tiled<4, RPT>), dim3((sf * W - 2 * M + 63) / 64,
                                                              (sf * H - 2 * M + 16 * RPT - 1) / (16 * RPT), B * 3),
                               dim3(256), lds, (hipStream_t)stream, q, gen, out, H, W, ph, w_up, kd, M);
    } else {
        const long long n = (long long)B * 3 * (sf * H - 2 * M) * (sf * W - 2 * M);
        hipLaunchKernelGGL(cem_up_add_kernel, dim3(nblocks(n)), dim3(NT), 0, (hipStream_t)stream, q, gen, out, B, H,
                           W, sf, ph, w_up, kd, M);
    }
    return launched();
}

extern "C" int esr_prep_input_s(const float *x, int32_t B, int32_t nz, int32_t h, int32_t w, int32_t sf, int32_t m,
                                float *lr_nchw, float *first, int32_t first_cp, int32_t first_lr_off,
                                float *const *zlr_dst, const int32_t *zlr_cp, int32_t n_zlr, float *const *zhr_dst,
                                const int32_t *zhr_cp, int32_t n_zhr, int32_t split, float act_scale,
                                esr_stream_t stream) {
    if (!x || B <= 0 || h <= 0 || w <= 0 || sf <= 0 || m < 0 || nz < 0 || n_zlr < 0 || n_zlr > 4 || n_zhr < 0 ||
        n_zhr > 4 || !(act_scale > 0.f))
        return ESR_EINVAL;
    PrepParams p = {};
    p.x = x; p.B = B; p.nz = nz; p.h = h; p.w = w; p.sf = sf; p.m = m; p.split = split; p.ascale = act_scale;
    p.lr_nchw = lr_nchw; p.first = first; p.first_cp = first_cp; p.first_lr_off = first_lr_off;
    p.n_zlr = nz ? n_zlr : 0;
    p.n_zhr = nz ? n_zhr : 0;
    for (int i = 0; i < p.n_zlr; ++i) { p.zlr[i] = zlr_dst[i]; p.zlr_cp[i] = zlr_cp[i]; }
    for (int i = 0; i < p.n_zhr; ++i) { p.zhr[i] = zhr_dst[i]; p.zhr_cp[i] = zhr_cp[i]; }
    const int H = h + 2 * m, W = w + 2 * m;
    hipLaunchKernelGGL(prep_lr_kernel, dim3(nblocks((long long)B * H * W)), dim3(NT), 0, (hipStream_t)stream, p);
    int rc = launched();
    if (rc || !p.n_zhr) return rc;
    hipLaunchKernelGGL(prep_hr_kernel, dim3(nblocks((long long)B * sf * H * sf * W)), dim3(NT), 0,
                       (hipStream_t)stream, p);
    return launched();
}

extern "C" int esr_prep_input(const float *x, int32_t B, int32_t nz, int32_t h, int32_t w, int32_t sf, int32_t m,
                              float *lr_nchw, float *first, int32_t first_cp, int32_t first_lr_off,
                              float *const *zlr_dst, const int32_t *zlr_cp, int32_t n_zlr, float *const *zhr_dst,
                              const int32_t *zhr_cp, int32_t n_zhr, int32_t split, esr_stream_t stream) {
    return esr_prep_input_s(x, B, nz, h, w, sf, m, lr_nchw, first, first_cp, first_lr_off, zlr_dst, zlr_cp, n_zlr,
                            zhr_dst, zhr_cp, n_zhr, split, 1.f, stream);
}
