// Probe of v_permlane32_swap's lane pairing (result printed; used to fix the x3 direct epilogue's operand order).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned *a) {
    const unsigned t = threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(t, 100u + t, false, false);
    a[t] = r[0];
    a[64 + t] = r[1];
}
int main() {
    unsigned *d, h[128];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("dst(after): lane0=%u lane31=%u lane32=%u lane63=%u\n", h[0], h[31], h[32], h[63]);
    printf("src(after): lane0=%u lane31=%u lane32=%u lane63=%u\n", h[64], h[95], h[96], h[127]);
    return 0;
}
