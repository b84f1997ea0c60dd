// Kernel-selection setters of the ablation library (esr_ablation.h).  Compiled into libesr_exp.so only: in the product
// library the knobs are compile-time constants (esr_knobs.h) and this file is empty.
#include "esr_amd.h"
#include "esr_knobs.h"

#ifdef ESR_X3_EXPERIMENTS
#include "esr_ablation.h"

#define ESR_KNOB_DEF(name, v) int name = v;
ESR_KNOBS(ESR_KNOB_DEF)
#undef ESR_KNOB_DEF

namespace {
int set_knob(int &knob, int32_t v, int lo, int hi) {
    if (v < lo || v > hi) return ESR_EINVAL;
    const int prev = knob;
    knob = v;
    return prev;
}
}  // namespace

extern "C" int esr_x3_set_kernel(int32_t variant) { return set_knob(g_x3_kernel, variant, 0, 88); }
extern "C" int esr_x3_set_tile_map(int32_t mode) { return set_knob(g_tile_map, mode, 0, 1); }
extern "C" int esr_x3_set_narrow(int32_t on) { return set_knob(g_x3_narrow, on, 0, 1); }
extern "C" int esr_x3_set_nsplit(int32_t on) { return set_knob(g_x3_nsplit, on, 0, 1); }
extern "C" int esr_conv_set_tile(int32_t rows) {
    if (rows != 0 && rows != 4 && rows != 8) return ESR_EINVAL;
    return set_knob(g_conv_tile, rows, 0, 8);
}
extern "C" int esr_cem_set_direct(int32_t direct) { return set_knob(g_cem_direct, direct, 0, 1); }
extern "C" int esr_wgrad_set_kernel(int32_t variant) { return set_knob(g_wgrad_kernel, variant, 0, 1); }
extern "C" int esr_wgrad3_set_dma(int32_t on) { return set_knob(g_wgrad3_dma, on, 0, 1); }
extern "C" int esr_wgrad3d_set_dbg(int32_t mode) { return set_knob(g_wgrad3d_dbg, mode, 0, 3); }
extern "C" int esr_wgrad3d_set_unroll(int32_t u) {
    if (u != 1 && u != 2 && u != 4) return ESR_EINVAL;
    return set_knob(g_wgrad3d_unroll, u, 1, 4);
}
extern "C" int esr_dconv_set_halo(int32_t on) { return set_knob(g_dconv_halo, on, 0, 2); }
extern "C" int esr_dconv_set_occ3(int32_t on) { return set_knob(g_dconv_occ3, on, 0, 1); }
extern "C" int esr_dconv_set_cw16(int32_t on) { return set_knob(g_dconv_cw16, on, 0, 1); }
extern "C" int esr_dconv_set_rows(int32_t on) { return set_knob(g_dconv_rows, on, 0, 1); }
extern "C" int esr_axpby_set_rows(int32_t on) { return set_knob(g_axpby_rows, on, 0, 2); }
extern "C" int esr_bn_set_onepass(int32_t on) { return set_knob(g_bn_onepass, on, 0, 1); }
#endif  // ESR_X3_EXPERIMENTS
