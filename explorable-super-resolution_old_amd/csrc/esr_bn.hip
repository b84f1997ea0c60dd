// esr_bn.hip — the discriminator's BatchNorm2d (training mode) + LeakyReLU pair of conv_block(CNA) (block.py:129-156,
// architecture.py:222-284) fused: forward, backward and the backward's own backward (the WGAN-GP penalty differentiates
// the D input gradient once more, loss.py:244-263).
//
// Tensors are the discriminator's channels-last activations: [P][C] fp32, P = B·H·W rows.  Per channel c:
//   μ = mean(x), v = mean((x − μ)²) (biased), r = (v + eps)^-1/2, x̂ = (x − μ)·r, z = γ·x̂ + β, y = z > 0 ? z : a·z.
// Backward (m = z > 0 ? 1 : a, gz = gy·m, N = P):
//   s1 = Σ gz (= dβ), s2 = Σ gz·x̂ (= dγ), gx = γ·r·(gz − s1/N − x̂·s2/N).
// Double backward of (x, γ, gy) -> (gx, dγ, dβ) given upstream (u, gg_γ, gg_β) (the mask is piecewise constant):
//   A = Σ u·x̂, U = Σ u, Q = Σ u·gz
//   g_gy = m·[γ·r·(u − U/N − x̂·A/N) + gg_γ·x̂ + gg_β]
//   g_γ  = r·(Q − s1·U/N − s2·A/N)
//   G_x̂  = −(γr/N)(u·s2 + A·gz) + gg_γ·gz            (∂/∂x̂ at fixed r)
//   G_r  = γ·(Q − s1·U/N − s2·A/N)                     (∂/∂r at fixed x̂)
//   g_x  = r·(G_x̂ − mean(G_x̂) − x̂·mean(G_x̂·x̂)) − G_r·r²·x̂/N,  with
//          mean(G_x̂) = −(γr/N)(s2·U + A·s1)/N + gg_γ·s1/N,  mean(G_x̂·x̂) = −2(γr/N)·s2·A/N + gg_γ·s2/N.
// Every pass is either a per-channel column reduction (block partials summed in a fixed order: deterministic) or one
// elementwise pass; z and the mask are recomputed from (x, μ, r, γ, β) by the same expression everywhere.  The column
// sums accumulate in float64 (per-thread, block and final), as PyTorch's own BatchNorm does on the CPU (acc_type<float>
// = double): the mean-removal terms then cancel to float64 rounding, not to that of float32 running sums.
#include <hip/hip_runtime.h>
#include "esr_amd.h"
#include "esr_knobs.h"

namespace {

constexpr int NT = 256;
constexpr int MAXB = 1024;  // partial-sum blocks per reduction

struct BnP {
    const float *x, *gy, *u;          // [P][C]
    const float *gamma, *beta;        // [C]
    const float *mu, *rs;             // [C] mean, 1/sqrt(var + eps)
    const float *sums;                // [5][C] per-channel sums of the previous reduction
    const float *ggg, *ggb;           // [C] upstream gradients of dγ / dβ, or null
    long long P;
    int C;
    float slope;
};

__device__ __forceinline__ float xhat_of(const BnP &p, float x, int c) { return (x - p.mu[c]) * p.rs[c]; }
__device__ __forceinline__ float mask_of(const BnP &p, float xh, int c) {
    const float z = p.gamma[c] * xh + p.beta[c];
    return z > 0.f ? 1.f : p.slope;
}

// Column reduction: mode 0: Σx; 1: Σ(x − μ)²; 2: Σgz, Σgz·x̂; 3: Σu, Σu·x̂, Σu·gz; 4: Σd, Σd² with d = x − x[0][c]
// (the forward's statistics in one pass: moments about the channel's first value, so the variance does not come from
// the difference of two large sums).  partial[block][k][C] (float64).
template <int MODE>
__global__ __launch_bounds__(NT) void bn_colsum(BnP p, double *partial) {
    constexpr int K = MODE == 3 ? 3 : ((MODE == 2 || MODE == 4) ? 2 : 1);
    __shared__ double red[K][NT];
    const int C = p.C, tid = threadIdx.x;
    // thread -> (channel c, row phase) for C <= NT; channel loop otherwise
    const int rpi = C <= NT ? NT / C : 1;  // rows per iteration
    const long long rows_per_block = (p.P + gridDim.x - 1) / gridDim.x;
    const long long r0 = (long long)blockIdx.x * rows_per_block;
    const long long r1 = min(p.P, r0 + rows_per_block);
    for (int cb = 0; cb < C; cb += NT) {
        const int c = C <= NT ? tid % C : cb + tid;
        const int ph = C <= NT ? tid / C : 0;
        const bool act = (C <= NT ? tid < rpi * C : c < C);
        double s[K];
#pragma unroll
        for (int k = 0; k < K; ++k) s[k] = 0.0;
        const double shift = (MODE == 4 && act) ? (double)p.x[c] : 0.0;
        if (act) {
#pragma unroll 4
            for (long long r = r0 + ph; r < r1; r += rpi) {
                const long long i = r * C + c;
                const float x = p.x[i];
                if (MODE == 0) {
                    s[0] += x;
                } else if (MODE == 4) {
                    const double d = (double)x - shift;
                    s[0] += d;
                    s[1] += d * d;
                } else if (MODE == 1) {
                    const double d = (double)x - (double)p.mu[c];
                    s[0] += d * d;
                } else {
                    const float xh = xhat_of(p, x, c);
                    const float gz = p.gy[i] * mask_of(p, xh, c);
                    if (MODE == 2) {
                        s[0] += gz;
                        s[1] += (double)gz * xh;
                    } else {
                        const float u = p.u[i];
                        s[0] += u;
                        s[1] += (double)u * xh;
                        s[2] += (double)u * gz;
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) red[k][tid] = s[k];
        __syncthreads();
        if (C <= NT) {
            if (tid < C)
                for (int k = 0; k < K; ++k) {
                    double v = 0.0;
                    for (int q = 0; q < rpi; ++q) v += red[k][q * C + tid];
                    partial[((long long)blockIdx.x * K + k) * C + tid] = v;
                }
        } else if (c < C) {
            for (int k = 0; k < K; ++k) partial[((long long)blockIdx.x * K + k) * C + c] = red[k][tid];
        }
        __syncthreads();
        if (C <= NT) break;
    }
}

// out[k][c] = Σ_b partial[b][k][c]: workgroup = 32 consecutive (k, c) outputs × 8 slices of the blocks, each slice
// summed in block order, then the slices in slice order (fixed order: deterministic)
template <typename T>
__global__ void bn_finish(const double *partial, int nblk, int K, int C, T *out) {
    __shared__ double sl[8][32];
    const int o = threadIdx.x & 31, q = threadIdx.x >> 5;
    const int i = blockIdx.x * 32 + o;
    const int b0 = nblk * q / 8, b1 = nblk * (q + 1) / 8;
    double v = 0.0;
    if (i < K * C) {
        const int k = i / C, c = i - k * C;
#pragma unroll 4
        for (int b = b0; b < b1; ++b) v += partial[((long long)b * K + k) * C + c];
    }
    sl[q][o] = v;
    __syncthreads();
    if (q == 0 && i < K * C) {
        double t = sl[0][o];
        for (int r = 1; r < 8; ++r) t += sl[r][o];
        out[i] = (T)t;
    }
}

// mean / invstd from the sums: mode 0 -> mu = s/N; mode 1 -> rs = 1/sqrt(s/N + eps) (and var = s/N), and, with rm
// set, nn.BatchNorm2d's running-buffer update (momentum m): rm = rm·(1 - m) + m·mu, rv = rv·(1 - m) + m·N/(N-1)·var,
// num_batches_tracked + 1 — in this launch instead of five PyTorch ops per layer and call
struct BnRun {
    float *rm, *rv;
    long long *nbt;
    float m;
};

__global__ void bn_stats_finish(const float *sum, int C, long long P, float eps, int mode, float *mu, float *rs,
                                float *var, BnRun run) {
    const int c = blockIdx.x * NT + threadIdx.x;
    if (c >= C) return;
    if (mode == 0) {
        mu[c] = sum[c] / (float)P;
    } else {
        const float v = sum[c] / (float)P;
        var[c] = v;
        rs[c] = 1.f / sqrtf(v + eps);
        if (run.rm) {
            const float m = run.m, a = m * (float)P / (float)(P > 1 ? P - 1 : 1);
            run.rm[c] = run.rm[c] * (1.f - m) + m * mu[c];
            run.rv[c] = run.rv[c] * (1.f - m) + a * v;
            if (c == 0 && run.nbt) run.nbt[0] += 1;
        }
    }
}

// mode 0: y = lrelu(z); 1: gx (sums = [Σgz, Σgz·x̂]); 2: g_x, g_gy (sums = [Σgz, Σgz·x̂, U, A, Q])
template <int MODE>
__global__ void bn_apply(BnP p, float *o1, float *o2) {
    const long long i = (long long)blockIdx.x * NT + threadIdx.x;
    if (i >= p.P * p.C) return;
    const int c = (int)(i % p.C);
    const float x = p.x[i];
    const float xh = xhat_of(p, x, c);
    const float g = p.gamma[c], r = p.rs[c];
    if (MODE == 0) {
        const float z = g * xh + p.beta[c];
        o1[i] = z > 0.f ? z : p.slope * z;
        return;
    }
    const float m = mask_of(p, xh, c);
    const float invN = 1.f / (float)p.P;
    const float s1 = p.sums[c], s2 = p.sums[p.C + c];
    const float gz = p.gy[i] * m;
    if (MODE == 1) {
        o1[i] = g * r * (gz - s1 * invN - xh * s2 * invN);
        return;
    }
    const float U = p.sums[2 * p.C + c], A = p.sums[3 * p.C + c], Q = p.sums[4 * p.C + c];
    const float ggg = p.ggg ? p.ggg[c] : 0.f, ggb = p.ggb ? p.ggb[c] : 0.f;
    const float u = p.u ? p.u[i] : 0.f;
    const float gr = g * r;
    // g_gy
    o2[i] = m * (gr * (u - U * invN - xh * A * invN) + ggg * xh + ggb);
    // g_x
    const float Gx = -(gr * invN) * (u * s2 + A * gz) + ggg * gz;
    const float mG = -(gr * invN) * (s2 * U + A * s1) * invN + ggg * s1 * invN;
    const float mGx = -2.f * (gr * invN) * s2 * A * invN + ggg * s2 * invN;
    const float Gr = g * (Q - s1 * U * invN - s2 * A * invN);
    o1[i] = r * (Gx - mG - xh * mGx) - Gr * r * r * xh * invN;
}

// mode 4's sums (float64) -> μ = x[0][c] + Σd/N, var = Σd²/N − (Σd/N)², rs and the running buffers as bn_stats_finish
__global__ void bn_stats_onepass(const double *sum, const float *x, int C, long long P, float eps, float *mu, float *rs,
                                 float *var, BnRun run) {
    const int c = blockIdx.x * NT + threadIdx.x;
    if (c >= C) return;
    const double m1 = sum[c] / (double)P, m2 = sum[C + c] / (double)P;
    const float m = (float)((double)x[c] + m1);
    const float v = (float)fmax(m2 - m1 * m1, 0.0);
    mu[c] = m;
    var[c] = v;
    rs[c] = 1.f / sqrtf(v + eps);
    if (run.rm) {
        const float mo = run.m, a = mo * (float)P / (float)(P > 1 ? P - 1 : 1);
        run.rm[c] = run.rm[c] * (1.f - mo) + mo * m;
        run.rv[c] = run.rv[c] * (1.f - mo) + a * v;
        if (c == 0 && run.nbt) run.nbt[0] += 1;
    }
}

// g_γ[c] = r·(Q − s1·U/N − s2·A/N)
__global__ void bn_ggamma(const float *sums, const float *rs, int C, long long P, float *out) {
    const int c = blockIdx.x * NT + threadIdx.x;
    if (c >= C) return;
    const float invN = 1.f / (float)P;
    const float s1 = sums[c], s2 = sums[C + c], U = sums[2 * C + c], A = sums[3 * C + c], Q = sums[4 * C + c];
    out[c] = rs[c] * (Q - s1 * U * invN - s2 * A * invN);
}

inline int launched() { return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH; }
inline unsigned grid_of(long long n) { return (unsigned)((n + NT - 1) / NT); }
inline int nblocks_for(long long P) { return (int)(P / 256 < 1 ? 1 : (P / 256 > MAXB ? MAXB : P / 256)); }

template <int MODE, typename T = float>
int colsum(const BnP &p, float *ws, T *out, hipStream_t st) {
    double *partial = reinterpret_cast<double *>(ws);
    constexpr int K = MODE == 3 ? 3 : ((MODE == 2 || MODE == 4) ? 2 : 1);
    const int nb = nblocks_for(p.P);
    hipLaunchKernelGGL(bn_colsum<MODE>, dim3(nb), dim3(NT), 0, st, p, partial);
    hipLaunchKernelGGL(bn_finish, dim3((unsigned)((K * p.C + 31) / 32)), dim3(NT), 0, st, partial, nb, K, p.C, out);
    return launched();
}

}  // namespace

extern "C" int esr_colsum(const float *x, int64_t P, int32_t C, float *out, float *ws, esr_stream_t stream) {
    if (!x || !out || !ws || P <= 0 || C <= 0) return ESR_EINVAL;
    BnP p{};
    p.x = x;
    p.P = P;
    p.C = C;
    return colsum<0>(p, ws, out, (hipStream_t)stream);
}

extern "C" int64_t esr_bn_workspace_floats(int64_t P, int32_t C) {
    return (int64_t)MAXB * 3 * C * 2 + 8LL * C;  // float64 partials, then [5][C] sums
}

extern "C" int esr_bn_lrelu_fwd(const float *x, int64_t P, int32_t C, const float *gamma, const float *beta, float eps,
                                float slope, float *y, float *mu, float *rs, float *var, float *ws,
                                float *running_mean, float *running_var, int64_t *num_batches_tracked, float momentum,
                                esr_stream_t stream) {
    if (!x || !gamma || !beta || !y || !mu || !rs || !var || !ws || P <= 0 || C <= 0) return ESR_EINVAL;
    if ((running_mean == nullptr) != (running_var == nullptr) || (running_mean && !(momentum >= 0.f && momentum <= 1.f)))
        return ESR_EINVAL;
    const BnRun run = {running_mean, running_var, reinterpret_cast<long long *>(num_batches_tracked), momentum};
    const BnRun none = {nullptr, nullptr, nullptr, 0.f};
    const hipStream_t st = (hipStream_t)stream;
    BnP p = {};
    p.x = x; p.gamma = gamma; p.beta = beta; p.mu = mu; p.rs = rs; p.P = P; p.C = C; p.slope = slope;
    float *partial = ws, *sums = ws + (long long)MAXB * 3 * C * 2;  // (room for [2][C] float64 sums: [8][C] floats)
    if (g_bn_onepass) {
        double *sd = reinterpret_cast<double *>(sums);
        if (colsum<4, double>(p, partial, sd, st)) return ESR_ELAUNCH;
        hipLaunchKernelGGL(bn_stats_onepass, dim3(grid_of(C)), dim3(NT), 0, st, sd, x, C, P, eps, mu, rs, var, run);
    } else {
        if (colsum<0>(p, partial, sums, st)) return ESR_ELAUNCH;
        hipLaunchKernelGGL(bn_stats_finish, dim3(grid_of(C)), dim3(NT), 0, st, sums, C, P, eps, 0, mu, rs, var, none);
        if (colsum<1>(p, partial, sums, st)) return ESR_ELAUNCH;
        hipLaunchKernelGGL(bn_stats_finish, dim3(grid_of(C)), dim3(NT), 0, st, sums, C, P, eps, 1, mu, rs, var, run);
    }
    hipLaunchKernelGGL(bn_apply<0>, dim3(grid_of(P * C)), dim3(NT), 0, st, p, y, nullptr);
    return launched();
}

extern "C" int esr_bn_lrelu_bwd(const float *x, const float *gy, int64_t P, int32_t C, const float *gamma,
                                const float *beta, const float *mu, const float *rs, float slope, float *gx,
                                float *sums2, float *ws, esr_stream_t stream) {
    if (!x || !gy || !gamma || !beta || !mu || !rs || !gx || !sums2 || !ws || P <= 0 || C <= 0) return ESR_EINVAL;
    const hipStream_t st = (hipStream_t)stream;
    BnP p = {};
    p.x = x; p.gy = gy; p.gamma = gamma; p.beta = beta; p.mu = mu; p.rs = rs; p.P = P; p.C = C; p.slope = slope;
    if (colsum<2>(p, ws, sums2, st)) return ESR_ELAUNCH;
    p.sums = sums2;
    hipLaunchKernelGGL(bn_apply<1>, dim3(grid_of(P * C)), dim3(NT), 0, st, p, gx, nullptr);
    return launched();
}

extern "C" int esr_bn_lrelu_bwd2(const float *x, const float *gy, const float *u, const float *ggg, const float *ggb,
                                 int64_t P, int32_t C, const float *gamma, const float *beta, const float *mu,
                                 const float *rs, float slope, const float *sums2, float *g_x, float *g_gy,
                                 float *g_gamma, float *ws, esr_stream_t stream) {
    if (!x || !gy || !gamma || !beta || !mu || !rs || !sums2 || !g_x || !g_gy || !g_gamma || !ws || P <= 0 || C <= 0)
        return ESR_EINVAL;
    const hipStream_t st = (hipStream_t)stream;
    BnP p = {};
    p.x = x; p.gy = gy; p.u = u; p.gamma = gamma; p.beta = beta; p.mu = mu; p.rs = rs; p.P = P; p.C = C;
    p.slope = slope; p.ggg = ggg; p.ggb = ggb;
    float *partial = ws, *sums5 = ws + (long long)MAXB * 3 * C * 2;  // [Σgz, Σgz·x̂, U, A, Q]
    (void)hipMemcpyAsync(sums5, sums2, 2 * C * sizeof(float), hipMemcpyDeviceToDevice, st);
    if (u) {
        if (colsum<3>(p, partial, sums5 + 2 * C, st)) return ESR_ELAUNCH;
    } else {
        (void)hipMemsetAsync(sums5 + 2 * C, 0, 3 * C * sizeof(float), st);
    }
    p.sums = sums5;
    hipLaunchKernelGGL(bn_apply<2>, dim3(grid_of(P * C)), dim3(NT), 0, st, p, g_x, g_gy);
    hipLaunchKernelGGL(bn_ggamma, dim3(grid_of(C)), dim3(NT), 0, st, sums5, rs, C, P, g_gamma);
    return launched();
}
