// esr_conv.hip — 3×3 convolution (and polyphase nearest-×2 upconv) for gfx950, fp32 via f32-input MFMA.
//
// Implicit GEMM: M = output pixels, N = output channels (32 or 64), K = taps × input channels.
// Workgroup = 256 threads (4 waves, one per SIMD), output tile TH×TW = 4·MT rows × 32 columns of one image, all N.
// Each wave owns MT tile rows (32-pixel M-tiles) × NT 32-channel N-tiles: MT·NT accumulators of
// v_mfma_f32_32x32x2_f32 (16 f32 per lane each).  MT = 2 by default; MT = 1 for small grids (see launch_conv).
// K loop: input channels in chunks of ≤32.  Per chunk the (TH+2)×(TW+2) halo tile of the chunk's channels and the
// chunk's packed weights [taps][N][32] are staged in LDS (pixel/row pitch 36 floats: 16-byte slots of the 32 lanes of a
// ds_read_b128 group land on 16 distinct slots); the next chunk is prefetched into registers while MFMAs run.
// K permutation inside a chunk: lane half h (lane>>5) consumes channels [h*kc/2, (h+1)*kc/2) four at a time with one
// ds_read_b128 for A (pixel) and one for B (weights); A and B use the same map so the sum is unchanged.
//
// Numerics: v_mfma_f32_32x32x2_f32 is an exact fp32 FMA chain (cdna_hip_programming.md §3), so results differ from
// a CPU fp32 conv only by summation order.
#include <hip/hip_runtime.h>
#include "esr_amd.h"
#include "esr_knobs.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// Tile: 4 waves × MT rows × 32 columns (MT = 2: 8×32, the default; MT = 1: 4×32 for grids that would otherwise
// leave the last round of workgroups mostly idle, and small enough in LDS for two workgroups per CU when N = 32).
constexpr int TW = 32, HX = TW + 2;
constexpr int KC = 32;
constexpr int PS = 36;  // LDS pitch (floats) of a staged pixel / weight row
constexpr int NTHREADS = 256;

struct ConvParams {
    const float *in;
    int B, H, W, in_cp, cin;
    const float *w;
    const float *bias;
    int cout;
    int tap_y0, tap_x0;  // halo-tile offset of tap 0 (0,0 for 3×3; (py,px) for an upconv phase)
    int tiles_x, tiles_y;
    int xcd_map;  // 1: XCD-grouped tile order
    esr_conv_out o;
};

template <int NT, int TS, int MT>
__global__ __launch_bounds__(NTHREADS, (MT == 1 && NT == 1) ? 2 : 1) void conv_fwd_kernel(ConvParams p) {
    constexpr int TH = 4 * MT, HY = TH + 2;
    constexpr int IN_F4 = HY * HX * (KC / 4);                    // float4s of a full input chunk
    constexpr int IN_ITERS = (IN_F4 + NTHREADS - 1) / NTHREADS;
    constexpr int T = TS * TS;
    constexpr int N = NT * 32;
    constexpr int W_F4 = T * N * (KC / 4);
    constexpr int W_ITERS = (W_F4 + NTHREADS - 1) / NTHREADS;
    __shared__ __attribute__((aligned(16))) float lds[HY * HX * PS + T * N * PS];
    float *s_in = lds;
    float *s_w = lds + HY * HX * PS;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int hl = lane >> 5;   // lane half
    const int ml = lane & 31;

    // XCD-grouped tile order (esr_x3_set_tile_map; same renumbering as esr_conv_x3.hip's xcd_tile): workgroup b runs on
    // XCD b % 8, and each XCD takes one contiguous run of tiles so neighbouring tiles share its L2
    int t = blockIdx.x;
    if (p.xcd_map) {
        const int nb = gridDim.x, x = t % 8, l = t / 8, q = nb / 8, r = nb % 8;
        t = x < r ? x * (q + 1) + l : r * (q + 1) + (x - r) * q + l;
    }
    const int tx = t % p.tiles_x;
    t /= p.tiles_x;
    const int ty = t % p.tiles_y;
    const int b = t / p.tiles_y;
    const int y0 = ty * TH, x0 = tx * TW;  // output tile origin; halo origin in padded coords is the same numbers

    const long long rowp = (long long)(p.W + 2);
    const float *in_b = p.in + (long long)b * (p.H + 2) * rowp * p.in_cp;
    const int nchunk = (p.cin + KC - 1) / KC;

    f32x4 rin[IN_ITERS];
    f32x4 rw[W_ITERS];

    auto load_chunk = [&](int j) {
        const int c0 = j * KC;
        const int kc = min(KC, p.cin - c0);
        const int kc4 = kc >> 2;
        const int cnt = HY * HX * kc4;
#pragma unroll
        for (int k = 0; k < IN_ITERS; ++k) {
            const int idx = tid + k * NTHREADS;
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (idx < cnt) {
                const int px = idx / kc4;
                const int c4 = idx - px * kc4;
                const int hy = px / HX, hx = px - (px / HX) * HX;
                const int gy = y0 + hy, gx = x0 + hx;  // padded coordinates
                if (gy < p.H + 2 && gx < p.W + 2)
                    v = *reinterpret_cast<const f32x4 *>(in_b + (gy * rowp + gx) * p.in_cp + c0 + c4 * 4);
            }
            rin[k] = v;
        }
        const float *wj = p.w + (long long)j * W_F4 * 4;
#pragma unroll
        for (int k = 0; k < W_ITERS; ++k) {
            const int idx = tid + k * NTHREADS;
            if (idx < W_F4) rw[k] = *reinterpret_cast<const f32x4 *>(wj + idx * 4);
        }
    };
    auto store_chunk = [&](int j) {
        const int kc = min(KC, p.cin - j * KC);
        const int kc4 = kc >> 2;
        const int cnt = HY * HX * kc4;
#pragma unroll
        for (int k = 0; k < IN_ITERS; ++k) {
            const int idx = tid + k * NTHREADS;
            if (idx < cnt) {
                const int px = idx / kc4;
                const int c4 = idx - px * kc4;
                *reinterpret_cast<f32x4 *>(s_in + px * PS + c4 * 4) = rin[k];
            }
        }
#pragma unroll
        for (int k = 0; k < W_ITERS; ++k) {
            const int idx = tid + k * NTHREADS;
            if (idx < W_F4) *reinterpret_cast<f32x4 *>(s_w + (idx >> 3) * PS + (idx & 7) * 4) = rw[k];
        }
    };

    f32x16 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
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
        const int kc = min(KC, p.cin - j * KC);
        const int half = kc >> 1;
        const int ngroups = kc >> 3;
#pragma unroll
        for (int tap = 0; tap < T; ++tap) {
            const int dy = p.tap_y0 + tap / TS, dx = p.tap_x0 + tap % TS;
            const float *a0 = s_in + ((MT * wave + dy) * HX + ml + dx) * PS + hl * half;
            const float *bw = s_w + (tap * N + ml) * PS + hl * half;
            for (int g = 0; g < ngroups; ++g) {
                f32x4 av[MT], bv[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) av[mt] = *reinterpret_cast<const f32x4 *>(a0 + mt * HX * PS + 4 * g);
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) bv[nt] = *reinterpret_cast<const f32x4 *>(bw + nt * 32 * PS + 4 * g);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            acc[mt][nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mt][s], bv[nt][s], acc[mt][nt], 0, 0, 0);
                }
            }
        }
    }

    // Epilogue. D layout (32x32 f32 MFMA): lane holds column n = lane&31 (output channel), rows (pixels)
    // m = (r&3) + 8*(r>>2) + 4*(lane>>5) for r = 0..15.
    const esr_conv_out &o = p.o;
    const long long orow = (long long)(o.out_w + 2);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int n = nt * 32 + ml;
        if (n >= p.cout) continue;
        const float bn = p.bias[n];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int y = y0 + MT * wave + mt;
            if (y >= p.H) continue;
            const int oy = o.out_sy * y + o.out_oy;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int x = x0 + (r & 3) + 8 * (r >> 2) + 4 * hl;
                if (x >= p.W) continue;
                const int ox = o.out_sx * x + o.out_ox;
                float v = acc[mt][nt][r] + bn;
                if (o.lrelu == 1) v = v > 0.f ? v : 0.2f * v;
                const long long pix = ((long long)b * (o.out_h + 2) + oy + 1) * orow + ox + 1;
                if (o.r1) v = o.s1 * v + o.r1[pix * o.r1_cp + o.r1_coff + n];
                if (o.lrelu == 2) {
                    v = o.r2[pix * o.r2_cp + o.r2_coff + n] > 0.f ? v : 0.2f * v;
                } else if (o.lrelu == 3) {  // the saved activation in the split-f16 layout
                    const _Float16 *g = reinterpret_cast<const _Float16 *>(
                        reinterpret_cast<const unsigned char *>(o.r2) + pix * o.r2_cp * 4 + ((o.r2_coff + n) >> 3) * 32);
                    const int e = (o.r2_coff + n) & 7;
                    v = ((float)g[e] + (float)g[8 + e]) > 0.f ? v : 0.2f * v;
                } else if (o.r2)
                    v = o.s2 * v + o.r2[pix * o.r2_cp + o.r2_coff + n];
                if (o.out_planar)
                    o.out[(((long long)b * p.cout + n) * o.out_h + oy) * o.out_w + ox] = v;
                else
                    o.out[pix * o.out_cp + o.out_coff + n] = v;
                if (o.out2) o.out2[pix * o.out2_cp + o.out2_coff + n] = v;
            }
        }
    }
}

int n_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0, v = 0;
        n = (hipGetDevice(&dev) == hipSuccess &&
             hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
    }
    return n;
}

int launch_conv(const float *in, int B, int H, int W, int in_cp, int cin, const float *w, const float *bias, int cout,
                int taps_side, int ty0, int tx0, const esr_conv_out *o, hipStream_t stream) {
    if (!in || !w || !bias || !o || !o->out) return ESR_EINVAL;
    if (B <= 0 || H <= 0 || W <= 0 || cin <= 0 || cout <= 0 || cout > 64) return ESR_EINVAL;
    if (cin % 8 || in_cp % 4 || in_cp < cin) return ESR_EINVAL;
    if (o->lrelu < 0 || o->lrelu > 3 || (o->lrelu >= 2 && !o->r2) || (o->lrelu == 3 && (o->r2_cp % 8 || o->r2_coff % 8)))
        return ESR_EINVAL;
    if (!o->out_planar && o->out_coff + cout > o->out_cp) return ESR_EINVAL;
    if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(w)) & 15) return ESR_EINVAL;
    ConvParams p;
    p.in = in; p.B = B; p.H = H; p.W = W; p.in_cp = in_cp; p.cin = cin;
    p.w = w; p.bias = bias; p.cout = cout; p.tap_y0 = ty0; p.tap_x0 = tx0;
    p.tiles_x = (W + TW - 1) / TW;
    // 4-row tiles for N = 32 (two workgroups per CU fit in LDS: measured 8-35 % faster, profiles/r1_conv_tile_ab.txt)
    // and for N = 64 when 8-row tiles would fill fewer than 8 rounds of one workgroup per CU (the last, partly idle
    // round then costs up to an eighth; at 8+ rounds the 8-row tile's better weight reuse wins); the ablation
    // library's esr_conv_set_tile overrides
    const int tiles8 = p.tiles_x * ((H + 7) / 8) * B;
    const int mt = g_conv_tile == 4 ? 1 : g_conv_tile == 8 ? 2 : ((cout <= 32 || tiles8 < 8 * n_cus()) ? 1 : 2);
    p.tiles_y = (H + 4 * mt - 1) / (4 * mt);
    p.xcd_map = g_tile_map;
    p.o = *o;
    const dim3 grid((unsigned)(p.tiles_x * p.tiles_y * B)), block(NTHREADS);
#define ESR_CONV_LAUNCH(NT_, TS_, MT_) hipLaunchKernelGGL((conv_fwd_kernel<NT_, TS_, MT_>), grid, block, 0, stream, p)
    if (mt == 1) {
        if (taps_side == 3) {
            if (cout > 32) ESR_CONV_LAUNCH(2, 3, 1); else ESR_CONV_LAUNCH(1, 3, 1);
        } else {
            if (cout > 32) ESR_CONV_LAUNCH(2, 2, 1); else ESR_CONV_LAUNCH(1, 2, 1);
        }
    } else {
        if (taps_side == 3) {
            if (cout > 32) ESR_CONV_LAUNCH(2, 3, 2); else ESR_CONV_LAUNCH(1, 3, 2);
        } else {
            if (cout > 32) ESR_CONV_LAUNCH(2, 2, 2); else ESR_CONV_LAUNCH(1, 2, 2);
        }
    }
#undef ESR_CONV_LAUNCH
    return hipGetLastError() == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

}  // namespace

extern "C" int esr_conv3x3_fwd(const float *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                               const float *w_packed, const float *bias, int32_t cout, const esr_conv_out *o,
                               esr_stream_t stream) {
    return launch_conv(in, B, H, W, in_cp, cin, w_packed, bias, cout, 3, 0, 0, o, (hipStream_t)stream);
}

extern "C" int esr_upconv2x_phase_fwd(const float *in, int32_t B, int32_t H, int32_t W, int32_t in_cp, int32_t cin,
                                      const float *w_packed, const float *bias, int32_t cout, int32_t py, int32_t px,
                                      const esr_conv_out *o, esr_stream_t stream) {
    if (py < 0 || py > 1 || px < 0 || px > 1) return ESR_EINVAL;
    return launch_conv(in, B, H, W, in_cp, cin, w_packed, bias, cout, 2, py, px, o, (hipStream_t)stream);
}

extern "C" int esr_abi_version(void) { return 23; }
