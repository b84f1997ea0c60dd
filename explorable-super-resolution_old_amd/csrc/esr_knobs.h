// Kernel-selection knobs of the launch functions.
//
// The product library (libesr_amd.so) has no mutable selection state: every knob below is a compile-time constant at
// its measured default, so which kernel a launch runs is a pure function of its arguments and the entry points of
// include/esr_amd.h are stateless and re-entrant across streams and threads.  The ablation library (`make exp`,
// -DESR_X3_EXPERIMENTS) turns them into process-wide variables behind the esr_*_set_* setters of esr_ablation.h (defined
// in esr_ablation.hip) for same-box A/B runs (tools/) and the variant-equality tests (tests/, `ablation_lib`).
#pragma once

// X(name, product value)
#define ESR_KNOBS(X)                                                                                                  \
    X(g_tile_map, 1)     /* XCD-grouped block -> tile order of the generator convs (0: row-major blockIdx)         */ \
    X(g_conv_tile, 0)    /* exact-fp32 conv tile rows: 0 automatic, 4 or 8                                         */ \
    X(g_x3_kernel, 1)    /* x3 conv kernel variant: 1 = automatic (include/esr_amd.h), others: esr_ablation.h      */ \
    X(g_x3_narrow, 1)    /* narrow-N kernel for HR_conv1 (cout <= 3, planar output)                                */ \
    X(g_x3_nsplit, 0)    /* N = 64 x3 convs on under-filled grids as two N = 32 launches (round 3; A/B only)       */ \
    X(g_cem_direct, 0)   /* the untiled CEM inverse / up-add kernels                                               */ \
    X(g_wgrad_kernel, 1) /* 1 = 12-wave weight-gradient kernel, 0 = 4-wave                                         */ \
    X(g_wgrad3_dma, 1)   /* x3 weight gradient of split-f16 output gradients on the LDS-DMA kernel                 */ \
    X(g_wgrad3d_unroll, 4) /* unroll of wgrad3d's K-block loop: 4 (full, round 6: 5-8 % faster), 2, 1; bitwise equal */ \
    X(g_wgrad3d_dbg, 0)  /* diagnostic time split of wgrad3d (garbage results): 1 LDS-DMA of the first tile only,  */ \
                         /* 2 no fragment reads / MFMAs, 3 both                                                    */ \
    X(g_dconv_halo, 1)   /* discriminator convs on the halo-tile kernels where they pay (0: gather; 2: wherever)   */ \
    X(g_dconv_cw16, 1)   /* x3 halo kernel with 16-column tiles on narrow grids                                    */ \
    X(g_dconv_occ3, 1)   /* x3 halo kernel at three workgroups per CU where its LDS allows                         */ \
    X(g_dconv_rows, 0)   /* tap-row discriminator weight-gradient kernel (slower at config 3)                      */ \
    X(g_axpby_rows, 2)   /* esr_axpby_gs: 1 row-walking kernel, 2 the same with 4 items in flight per thread, 0 one */ \
                         /* thread per 8-channel group                                                            */ \
    X(g_bn_onepass, 1)   /* BatchNorm forward statistics in one pass (shifted moments; 0: mean, then Σ(x − μ)²)    */

#ifdef ESR_X3_EXPERIMENTS
#define ESR_KNOB_DECL(name, v) extern int name;
#else
#define ESR_KNOB_DECL(name, v) constexpr int name = v;
#endif
ESR_KNOBS(ESR_KNOB_DECL)
#undef ESR_KNOB_DECL
