/*
 * esr_ablation.h — extra entry points of the ABLATION library (libesr_exp.so: `make exp`, -DESR_X3_EXPERIMENTS).
 *
 * Not part of the product ABI (include/esr_amd.h): the product library exports none of these and holds no kernel-
 * selection state.  The ablation library is built from the same sources; it exports the whole product ABI plus the
 * process-wide kernel-selection setters below (esr_knobs.h), the non-default kernel variants they reach, and the
 * diagnostic time-split variants (garbage outputs).  Used by tools/ (same-box A/B runs, time splits) and by the
 * variant-equality tests (tests/conftest.py `ablation_lib`).  Every setter returns the previous setting, or
 * ESR_EINVAL for an out-of-range value.
 */
#ifndef ESR_ABLATION_H
#define ESR_ABLATION_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* esr_conv3x3_fwd_x3 / esr_upconv2x_phase_fwd_x3 kernel (0..88; 65 = 12-column tiles for N = 64 too, two per CU; 70-84 the persistent kernel and the time-split ablations; 85 / 86 = N = 32 3x3 convs in 18 / 24-column tiles at two per CU, 87 = the 12-column kernel with per-chunk s_memrealtime stamps (esr_x3c_set_stamps), 88 = N = 32 3x3 convs on the 8-channel double-buffered kernel (not bitwise equal: another summation order); everything else automatic).  All non-diagnostic variants are bitwise identical.
 * 0 / 1 / 63 = automatic (the product dispatch); 24 = the round-1 automatic choice (classic kernel only: 8-row at three
 *   per CU or 16-row at two; 25 / 26 force one); 50 = column-tile kernel (16 columns); 60 = column tiles with the
 *   weights read into registers from global memory; 61 = 8 waves of 2 columns; 62 = weights copied to registers per
 *   chunk; 64 = 12-column tiles at three workgroups per CU;
 * 22 = classic with two LDS stages and one workgroup per CU; 23 = cout > 32 with 8-row tiles at two workgroups per CU;
 *   21 = prefetch distance 1; 20 = compiler-scheduled fragment reads; 27 / 28 = register epilogue (16- / 8-row);
 * 2 = ring kernel; 15 = ring with staggered DMA issue; 18 = ring with compiler-scheduled reads; 16 / 17 = persistent
 *   ring;
 * diagnostics (garbage outputs): 3-14, 19 (ring), 29-30, 40-46 (classic), 51-54 (column tiles), 55-59 (warp-
 *   specialised persistent form). */
int esr_x3_set_kernel(int32_t variant);
/* Variant 87's stamp buffer: 38 u64 per workgroup (kernel start, per K chunk before DMA / after its wait / after
 * compute, end); NULL: not stored.  Returns 0, or -1. */
int esr_x3c_set_stamps(void *buf);
/* Block -> tile order of the x3 and exact-fp32 generator convs: 1 = XCD-grouped (product), 0 = row-major. */
int esr_x3_set_tile_map(int32_t mode);
/* HR_conv1 on the narrow-N kernel: 1 (product) / 0 = N = 32 tiles (equal to the x3 rounding, not bitwise). */
int esr_x3_set_narrow(int32_t on);
/* N split of under-filled N = 64 x3 convs (round 3): 0 (product) / 1 = two N = 32 launches (bitwise identical). */
int esr_x3_set_nsplit(int32_t on);
/* esr_axpby_gs: 2 = row-walking kernel with 4 items in flight per thread (product), 1 = one item, 0 = one thread per
 * 8-channel group (round 3). */
int esr_axpby_set_rows(int32_t on);
/* BatchNorm forward statistics: 1 (product) = one pass of shifted moments, 0 = mean, then Σ(x − μ)² (round 2-5). */
int esr_bn_set_onepass(int32_t on);
/* Exact-fp32 conv tile rows: 0 (product: automatic), 4 or 8 (identical results). */
int esr_conv_set_tile(int32_t rows);
/* CEM stencils: 0 (product: LDS-tiled / register-window) / 1 = the direct kernels. */
int esr_cem_set_direct(int32_t direct);
/* esr_conv3x3_wgrad: 1 (product) = 12-wave kernel, 0 = 4-wave kernel (different summation order). */
int esr_wgrad_set_kernel(int32_t variant);
/* x3 weight gradient of split-f16 output gradients: 1 (product) = LDS-DMA kernel, 0 = register-staged kernel. */
int esr_wgrad3_set_dma(int32_t on);
/* Diagnostic time split of the LDS-DMA x3 weight-gradient kernel (garbage results): 0 (product), 1 = LDS-DMA of the
 * first pixel tile only, 2 = no fragment reads / MFMAs, 3 = both (loop skeleton). */
int esr_wgrad3d_set_dbg(int32_t mode);
/* Unroll of the LDS-DMA x3 weight-gradient kernel's K-block loop: 4 (product, full), 2 or 1 (bitwise identical). */
int esr_wgrad3d_set_unroll(int32_t u);
/* Discriminator convs: 1 (product) = halo-tile kernels where they pay, 0 = gather kernels, 2 = halo wherever it fits. */
int esr_dconv_set_halo(int32_t on);
/* x3 halo kernel at three workgroups per CU where its LDS allows: 1 (product) / 0 (bitwise identical). */
int esr_dconv_set_occ3(int32_t on);
/* x3 halo kernel with 16-column tiles on narrow grids: 1 (product) / 0 = the gather kernel there. */
int esr_dconv_set_cw16(int32_t on);
/* Split-precision discriminator weight gradient on the tap-row kernel: 0 (product) / 1. */
int esr_dconv_set_rows(int32_t on);

#ifdef __cplusplus
}
#endif
#endif /* ESR_ABLATION_H */
