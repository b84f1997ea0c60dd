// esr_conv_x3.hip — 3×3 convolution / polyphase upconv on f16 matrix cores with fp32-level accuracy ("x3" path).
//
// Every fp32 value v is carried as an f16 pair (hi = f16(v), lo = f16(v - hi)), |v - hi - lo| <= 2^-22 |v| (absolute
// 2^-25 below the f16 normal range).  A product a·b is evaluated as a_hi·b_hi + a_hi·b_lo + a_lo·b_hi on
// v_mfma_f32_32x32x16_f16 with fp32 accumulation; the dropped a_lo·b_lo term is <= 2^-22 |ab|.  Three f16 MFMAs
// (3 × 32 cycles per 32×32×16 block) replace eight f32 MFMAs (8 × 64 cycles per 32×32×16): 5.3× the MFMA throughput
// of the exact-fp32 path (esr_conv.hip) at ~1e-6 relative error.
//
// "Split" activation layout (include/esr_amd.h): per pixel, channels in groups of 8, each group 32 bytes =
// 8 × f16 hi then 8 × f16 lo.  Same 4 bytes per channel as fp32, so HBM traffic is unchanged, and the producer's
// epilogue writes the split form once instead of every consumer splitting it again.
// Weights: packed [chunk][tap][n_pad][32 channels as 4 split groups] (128 B per (tap, n)), pre-scaled by a power of
// two (w_scale) so their lo parts stay normal; the epilogue multiplies by 1/w_scale (exact).
//
// Workgroup: 256 threads (4 waves), output tile 8 rows × 32 cols, all N.  Wave w owns rows {2w, 2w+1} (two 32-pixel
// M-tiles) × NT 32-channel N-tiles.  Per 32-channel K chunk the halo tile (10×34 pixels × 128 B) and the chunk's
// weights are copied to LDS at a 144-byte pitch (9 16-byte slots: the 16 lanes of a ds_read_b128 group hit 16 distinct
// slots), the next chunk is prefetched into registers while the MFMAs run.  MFMA K-step s of a chunk: lane half h
// consumes channel group 2s+h (its 8 channels are the fragment's 8 K elements): one ds_read_b128 per plane per operand.
// Epilogue: accumulators are re-staged through LDS as fp32 [pixel][channel] so each thread finishes whole 8-channel
// groups: bias, LeakyReLU, residuals (split inputs), split + 16-byte stores, fp32 planar stores for the CEM input.
#include <hip/hip_runtime.h>
#include "esr_amd.h"

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int TH = 8, TW = 32, HY = TH + 2, HX = TW + 2;
constexpr int PIXB = 144;  // LDS bytes per staged pixel / weight row: 128 data + 16 pad
constexpr int NTHR = 256;
constexpr int IN_PIECES = HY * HX * 8;  // 16-byte pieces of a full 32-channel input chunk
constexpr int IN_IT = (IN_PIECES + NTHR - 1) / NTHR;

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

// load one split 8-channel group (32 B) and reconstruct fp32
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

template <int NT, int TS>
__global__ __launch_bounds__(NTHR, 1) void conv_x3_kernel(X3Params p) {
    constexpr int T = TS * TS;
    constexpr int N = NT * 32;
    constexpr int IN_BYTES = HY * HX * PIXB;
    constexpr int W_PIECES = T * N * 8;
    constexpr int W_IT = (W_PIECES + NTHR - 1) / NTHR;
    constexpr int EP_P = N + 4;  // fp32 pitch of the epilogue tile
    constexpr int MAIN_BYTES = IN_BYTES + T * N * PIXB;
    constexpr int EP_BYTES = TH * TW * EP_P * 4;
    constexpr int LDS_BYTES = MAIN_BYTES > EP_BYTES ? MAIN_BYTES : EP_BYTES;
    __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
    unsigned char *s_in = lds;
    unsigned char *s_w = lds + IN_BYTES;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int hl = lane >> 5;
    const int ml = lane & 31;

    int t = blockIdx.x;
    const int tx = t % p.tiles_x;
    t /= p.tiles_x;
    const int ty = t % p.tiles_y;
    const int b = t / p.tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;

    const long long rowp = (long long)(p.W + 2);
    const long long pixb = 4LL * p.in_cp;  // bytes per pixel
    const unsigned char *in_b = p.in + (long long)b * (p.H + 2) * rowp * pixb;
    const int nchunk = (p.cin + 31) / 32;

    u32x4 rin[IN_IT];
    u32x4 rw[W_IT];

    auto load_chunk = [&](int j) {
        const int kc = min(32, p.cin - 32 * j);
        const int kc16 = (kc + 15) & ~15;
        const int sh = kc16 == 32 ? 3 : 2;  // log2(pieces per pixel)
        const int real = kc >> 2;           // real pieces per pixel (kc*4 bytes / 16)
        const int cnt = HY * HX << sh;
        const unsigned char *base = in_b + 128LL * j;
#pragma unroll
        for (int k = 0; k < IN_IT; ++k) {
            const int idx = tid + k * NTHR;
            u32x4 v = {0u, 0u, 0u, 0u};
            if (idx < cnt) {
                const int px = idx >> sh;
                const int pc = idx & ((1 << sh) - 1);
                const int hy = px / HX, hx = px - hy * HX;
                const int gy = y0 + hy, gx = x0 + hx;
                if (pc < real && gy < p.H + 2 && gx < p.W + 2)
                    v = *reinterpret_cast<const u32x4 *>(base + (gy * rowp + gx) * pixb + pc * 16);
            }
            rin[k] = v;
        }
        const unsigned char *wj = p.w + (long long)j * W_PIECES * 16;
#pragma unroll
        for (int k = 0; k < W_IT; ++k) {
            const int idx = tid + k * NTHR;
            if (idx < W_PIECES) rw[k] = *reinterpret_cast<const u32x4 *>(wj + idx * 16);
        }
    };
    auto store_chunk = [&](int j) {
        const int kc = min(32, p.cin - 32 * j);
        const int kc16 = (kc + 15) & ~15;
        const int sh = kc16 == 32 ? 3 : 2;
        const int cnt = HY * HX << sh;
#pragma unroll
        for (int k = 0; k < IN_IT; ++k) {
            const int idx = tid + k * NTHR;
            if (idx < cnt)
                *reinterpret_cast<u32x4 *>(s_in + (idx >> sh) * PIXB + (idx & ((1 << sh) - 1)) * 16) = rin[k];
        }
#pragma unroll
        for (int k = 0; k < W_IT; ++k) {
            const int idx = tid + k * NTHR;
            if (idx < W_PIECES) *reinterpret_cast<u32x4 *>(s_w + (idx >> 3) * PIXB + (idx & 7) * 16) = rw[k];
        }
    };

    f32x16 acc[2][NT];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[mt][nt][r] = 0.f;

    load_chunk(0);
    for (int j = 0; j < nchunk; ++j) {
        __syncthreads();
        store_chunk(j);
        __syncthreads();
        if (j + 1 < nchunk) load_chunk(j + 1);
        const int kc = min(32, p.cin - 32 * j);
        const int nsteps = (kc + 15) >> 4;
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int dy = p.tap_y0 + tap / TS, dx = p.tap_x0 + tap % TS;
            const unsigned char *a0 = s_in + ((2 * wave + dy) * HX + ml + dx) * PIXB + hl * 32;
            const unsigned char *bw = s_w + (tap * N + ml) * PIXB + hl * 32;
            for (int s = 0; s < nsteps; ++s) {
                f16x8 ah[2], al[2], bh[NT], bl[NT];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    ah[mt] = *reinterpret_cast<const f16x8 *>(a0 + mt * HX * PIXB + s * 64);
                    al[mt] = *reinterpret_cast<const f16x8 *>(a0 + mt * HX * PIXB + s * 64 + 16);
                }
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    bh[nt] = *reinterpret_cast<const f16x8 *>(bw + nt * 32 * PIXB + s * 64);
                    bl[nt] = *reinterpret_cast<const f16x8 *>(bw + nt * 32 * PIXB + s * 64 + 16);
                }
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) {
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
                    }
            }
        }
    }

    // ---- epilogue: restage fp32 accumulators as [pixel][channel] ----
    __syncthreads();
    float *s_ep = reinterpret_cast<float *>(lds);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int pix = (2 * wave + mt) * TW + (r & 3) + 8 * (r >> 2) + 4 * hl;
                s_ep[pix * EP_P + nt * 32 + ml] = acc[mt][nt][r];
            }
    __syncthreads();

    const esr_conv_out &o = p.o;
    const long long orow = (long long)(o.out_w + 2);
    constexpr int GROUPS = N / 8;
    bool ok = true;
    for (int u = tid; u < TH * TW * GROUPS; u += NTHR) {
        const int pix = u / GROUPS, g = u - (u / GROUPS) * GROUPS;
        const int c = 8 * g;
        if (c >= p.cout) continue;
        const int y = y0 + pix / TW, x = x0 + pix % TW;
        if (y >= p.H || x >= p.W) continue;
        const int oy = o.out_sy * y + o.out_oy, ox = o.out_sx * x + o.out_ox;
        const long long opix = ((long long)b * (o.out_h + 2) + oy + 1) * orow + ox + 1;
        float v[8];
        const f32x4 v0 = *reinterpret_cast<const f32x4 *>(s_ep + pix * EP_P + c);
        const f32x4 v1 = *reinterpret_cast<const f32x4 *>(s_ep + pix * EP_P + c + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { v[j] = v0[j]; v[j + 4] = v1[j]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float bj = (c + j < p.cout) ? p.bias[c + j] : 0.f;
            v[j] = v[j] * p.w_scale_inv + bj;
            if (o.lrelu) v[j] = lrelu(v[j]);
        }
        if (o.r1) {
            float r[8];
            load_group(reinterpret_cast<const unsigned char *>(o.r1) + (opix * o.r1_cp + o.r1_coff + c) * 4, r);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = o.s1 * v[j] + r[j];
        }
        if (o.r2) {
            float r[8];
            load_group(reinterpret_cast<const unsigned char *>(o.r2) + (opix * o.r2_cp + o.r2_coff + c) * 4, r);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = o.s2 * v[j] + r[j];
        }
        if (o.out_planar) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (c + j < p.cout) o.out[(((long long)b * p.cout + c + j) * o.out_h + oy) * o.out_w + ox] = v[j];
        } else {
            ok &= store_group(reinterpret_cast<unsigned char *>(o.out) + (opix * o.out_cp + o.out_coff + c) * 4, v);
            if (o.out2) store_group(reinterpret_cast<unsigned char *>(o.out2) + (opix * o.out2_cp + o.out2_coff + c) * 4, v);
        }
    }
    if (!ok && p.overflow) atomicOr(p.overflow, 1);
}

int launch_x3(const void *in, int B, int H, int W, int in_cp, int cin, const void *w, const float *bias,
              float w_scale, int cout, int taps_side, int ty0, int tx0, const esr_conv_out *o, int *overflow,
              hipStream_t stream) {
    if (!in || !w || !bias || !o || !o->out) return ESR_EINVAL;
    if (B <= 0 || H <= 0 || W <= 0 || cin <= 0 || cout <= 0 || cout > 64 || !(w_scale > 0.f)) return ESR_EINVAL;
    if (cin % 8 || in_cp % 8 || in_cp < cin) return ESR_EINVAL;
    if (!o->out_planar && (cout % 8 || o->out_cp % 8 || o->out_coff % 8 || o->out_coff + cout > o->out_cp))
        return ESR_EINVAL;
    if ((o->r1 && (o->r1_cp % 8 || o->r1_coff % 8)) || (o->r2 && (o->r2_cp % 8 || o->r2_coff % 8)) ||
        (o->out2 && (o->out2_cp % 8 || o->out2_coff % 8)))
        return ESR_EINVAL;
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(w)) & 15) return ESR_EINVAL;
    X3Params p;
    p.in = static_cast<const unsigned char *>(in);
    p.B = B; p.H = H; p.W = W; p.in_cp = in_cp; p.cin = cin;
    p.w = static_cast<const unsigned char *>(w);
    p.bias = bias; p.w_scale_inv = 1.f / w_scale; p.cout = cout;
    p.tap_y0 = ty0; p.tap_x0 = tx0;
    p.tiles_x = (W + TW - 1) / TW;
    p.tiles_y = (H + TH - 1) / TH;
    p.overflow = overflow;
    p.o = *o;
    const dim3 grid((unsigned)(p.tiles_x * p.tiles_y * B)), block(NTHR);
    if (taps_side == 3) {
        if (cout > 32) hipLaunchKernelGGL((conv_x3_kernel<2, 3>), grid, block, 0, stream, p);
        else hipLaunchKernelGGL((conv_x3_kernel<1, 3>), grid, block, 0, stream, p);
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
