// esr_plan.hip — host-side op-list executor: replays a whole generator (+CEM) forward, built once by the Python layer
// as an array of esr_op records, in ONE call through the binding (no per-launch ctypes/Python round trip), with
// optional per-op HIP-event timing for the benchmark's per-kernel roofline.
#include <hip/hip_runtime.h>
#include <new>
#include "esr_amd.h"

namespace {

struct Timer {
    int n;
    hipEvent_t *ev;
};

int dispatch(const esr_op &op, hipStream_t s) {
    const void *const *p = op.p;
    const int32_t *i = op.i;
    esr_stream_t st = (esr_stream_t)s;
    switch (op.kind) {
    case ESR_OP_CONV3X3:
        return esr_conv3x3_fwd((const float *)p[0], i[0], i[1], i[2], i[3], i[4], (const float *)p[1],
                               (const float *)p[2], i[5], &op.o, st);
    case ESR_OP_CONV3X3_X3:
        return esr_conv3x3_fwd_x3(p[0], i[0], i[1], i[2], i[3], i[4], p[1], (const float *)p[2], op.f[0], i[5], &op.o,
                                  (int32_t *)p[3], st);
    case ESR_OP_UPCONV:
        return esr_upconv2x_phase_fwd((const float *)p[0], i[0], i[1], i[2], i[3], i[4], (const float *)p[1],
                                      (const float *)p[2], i[5], i[6], i[7], &op.o, st);
    case ESR_OP_UPCONV_X3:
        return esr_upconv2x_phase_fwd_x3(p[0], i[0], i[1], i[2], i[3], i[4], p[1], (const float *)p[2], op.f[0], i[5],
                                         i[6], i[7], &op.o, (int32_t *)p[3], st);
    case ESR_OP_PREP: {
        float *zlr[4] = {(float *)p[3], (float *)p[4], (float *)p[5], (float *)p[6]};
        float *zhr[2] = {(float *)p[7], (float *)p[8]};
        const int32_t zlr_cp[4] = {i[8], i[9], i[10], i[11]};
        const int32_t zhr_cp[2] = {i[13], i[14]};
        return esr_prep_input_s((const float *)p[0], i[0], i[1], i[2], i[3], i[4], i[5], (float *)p[1],
                                (float *)p[2], i[6], i[7], zlr, zlr_cp, i[12], zhr, zhr_cp, i[15], i[16],
                                op.f[0] > 0.f ? op.f[0] : 1.f, st);
    }
    case ESR_OP_CEM_DOWN:
        return esr_cem_down((const float *)p[0], (const float *)p[1], (float *)p[2], i[0], i[1], i[2], i[3], i[4],
                            (const float *)p[3], i[5], i[6], st);
    case ESR_OP_CEM_INV:
        return esr_cem_inv((const float *)p[0], (float *)p[1], i[0], i[1], i[2], (const float *)p[2], i[3], st);
    case ESR_OP_CEM_UP_ADD:
        return esr_cem_up_add((const float *)p[0], (const float *)p[1], (float *)p[2], i[0], i[1], i[2], i[3], i[4],
                              (const float *)p[3], i[5], i[6], st);
    case ESR_OP_HR_CONVS_X3:
        return esr_hr_convs_x3(p[0], i[0], i[1], i[2], i[3], i[4], p[1], (const float *)p[2], op.f[0], p[3],
                               (float *)p[4], (int32_t *)p[5], st);
    case ESR_OP_HR1_SUM:
        return esr_hr1_sum((const float *)p[0], i[0], i[1], i[2], (const float *)p[1], op.f[0], (float *)p[2], st);
    default:
        return ESR_EINVAL;
    }
}

}  // namespace

extern "C" esr_timer_t esr_timer_create(int32_t n_ops) {
    if (n_ops <= 0) return nullptr;
    Timer *t = new (std::nothrow) Timer;
    if (!t) return nullptr;
    t->n = n_ops;
    t->ev = new (std::nothrow) hipEvent_t[n_ops + 1];
    if (!t->ev) {
        delete t;
        return nullptr;
    }
    for (int k = 0; k <= n_ops; ++k)
        if (hipEventCreate(&t->ev[k]) != hipSuccess) {
            for (int j = 0; j < k; ++j) (void)hipEventDestroy(t->ev[j]);
            delete[] t->ev;
            delete t;
            return nullptr;
        }
    return t;
}

extern "C" int esr_timer_elapsed(esr_timer_t timer, float *ms) {
    Timer *t = static_cast<Timer *>(timer);
    if (!t || !ms) return ESR_EINVAL;
    if (hipEventSynchronize(t->ev[t->n]) != hipSuccess) return ESR_ELAUNCH;
    for (int k = 0; k < t->n; ++k)
        if (hipEventElapsedTime(&ms[k], t->ev[k], t->ev[k + 1]) != hipSuccess) return ESR_ELAUNCH;
    return ESR_OK;
}

extern "C" int esr_timer_record(esr_timer_t timer, int32_t k, esr_stream_t stream) {
    Timer *t = static_cast<Timer *>(timer);
    if (!t || k < 0 || k > t->n) return ESR_EINVAL;
    return hipEventRecord(t->ev[k], (hipStream_t)stream) == hipSuccess ? ESR_OK : ESR_ELAUNCH;
}

extern "C" int esr_timer_stamps(esr_timer_t timer, esr_timer_t ref, float *t_ms) {
    Timer *t = static_cast<Timer *>(timer), *r = static_cast<Timer *>(ref);
    if (!t || !r || !t_ms) return ESR_EINVAL;
    if (hipEventSynchronize(t->ev[t->n]) != hipSuccess) return ESR_ELAUNCH;
    for (int k = 0; k <= t->n; ++k)
        if (hipEventElapsedTime(&t_ms[k], r->ev[0], t->ev[k]) != hipSuccess) return ESR_ELAUNCH;
    return ESR_OK;
}

extern "C" void esr_timer_destroy(esr_timer_t timer) {
    Timer *t = static_cast<Timer *>(timer);
    if (!t) return;
    for (int k = 0; k <= t->n; ++k) (void)hipEventDestroy(t->ev[k]);
    delete[] t->ev;
    delete t;
}

extern "C" int esr_run_ops(const esr_op *ops, int32_t n, esr_timer_t timer, esr_stream_t stream) {
    if (!ops || n <= 0) return ESR_EINVAL;
    Timer *t = static_cast<Timer *>(timer);
    if (t && t->n != n) return ESR_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    for (int k = 0; k < n; ++k) {
        if (t && hipEventRecord(t->ev[k], s) != hipSuccess) return ESR_ELAUNCH;
        const int rc = dispatch(ops[k], s);
        if (rc != ESR_OK) return rc;
    }
    if (t && hipEventRecord(t->ev[n], s) != hipSuccess) return ESR_ELAUNCH;
    return ESR_OK;
}

extern "C" int esr_op_size(void) { return (int)sizeof(esr_op); }
