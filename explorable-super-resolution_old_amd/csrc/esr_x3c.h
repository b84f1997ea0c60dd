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
};

// taps_side 3: 3x3 conv (tap_y0 = tap_x0 = 0); 2: one polyphase phase of the nearest-x2 upconv (tap origin py, px)
int x3c_launch(const X3cParams &p, int taps_side, hipStream_t stream, int dbg = 0);
// warp-specialised persistent form (one workgroup per CU: 8 compute + 4 LDS-DMA loader waves, register epilogue)
int x3s_launch(const X3cParams &p, int taps_side, hipStream_t stream, int dbg = 0);
