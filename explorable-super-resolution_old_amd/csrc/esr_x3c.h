// esr_x3c.h — internal interface of the column-tile x3 conv kernel (esr_conv_x3c.hip), used by esr_conv_x3.hip.
#pragma once
#include <hip/hip_runtime.h>
#include "esr_amd.h"

struct X3cParams {
    const unsigned char *in;
    int B, H, W, in_cp, cin;
    const unsigned char *w;
    const float *bias;
    float w_scale_inv;
    int cout;
    int tap_y0, tap_x0, tiles_x, tiles_y;
    int xcd_map;
    int *overflow;
    esr_conv_out o;
    // weight source layout (0 = the kernel's own: N records per tap, T·N records per chunk): w_ld records per tap,
    // starting at record w_roff of each tap, w_cstride bytes per chunk — an N = 32 launch over one half of an N = 64
    // packing (launch_x3's N split)
    int w_ld, w_roff;
    long long w_cstride;
    // fused HR_conv1 (x3c_launch_hr1 only): this conv (HR_conv0, cout 64, LeakyReLU) stores no activations; its
    // epilogue writes HR_conv1's 27 per-tap partial products of every pixel into y1 (pitch 32 floats) instead, from
    // HR_conv1's x3-packed weights w1 (n_pad 32) over [the input's zc-channel latent slot | the 64 activations]
    const unsigned char *w1;
    float *y1;
    int zc1;
};

// taps_side 3: 3x3 conv (tap_y0 = tap_x0 = 0); 2: one polyphase phase of the nearest-x2 upconv (tap origin py, px)
int x3c_launch(const X3cParams &p, int taps_side, hipStream_t stream, int dbg = 0);
// warp-specialised persistent form (one workgroup per CU: 8 compute + 4 LDS-DMA loader waves, register epilogue)
int x3s_launch(const X3cParams &p, int taps_side, hipStream_t stream, int dbg = 0);
// N = 32 3×3 conv on the persistent double-buffered kernel (esr_conv_x3p.hip; cout <= 32, not planar)
int x3p_launch(const X3cParams &p, hipStream_t stream, int dbg = 0);
// HR_conv0 with HR_conv1's partial products as its only output (p.w1, p.y1, p.zc1; N = 64, 3×3, one launch)
int x3c_launch_hr1(const X3cParams &p, hipStream_t stream);
// out NCHW [B][3][H][W] = sinv · Σ_t y[b][y + ty][x + tx][3t + o] + bias[o] (y: padded [B][H+2][W+2][32], zero halo)
int hr1_sum_launch(const float *y, int B, int H, int W, const float *bias, float sinv, float *out, hipStream_t st);
