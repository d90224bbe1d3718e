// prints what the gfx950 permlane16/32 swap builtins return for lane ids
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
    const unsigned a = threadIdx.x;
    const auto r16 = __builtin_amdgcn_permlane16_swap(a, a, false, false);
    const auto r32 = __builtin_amdgcn_permlane32_swap(a, a, false, false);
    out[threadIdx.x * 4 + 0] = r16[0];
    out[threadIdx.x * 4 + 1] = r16[1];
    out[threadIdx.x * 4 + 2] = r32[0];
    out[threadIdx.x * 4 + 3] = r32[1];
}
int main() {
    unsigned* d; unsigned h[256];
    hipMalloc(&d, sizeof(h));
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l += 8) printf("lane %2d: p16 (%2u,%2u) p32 (%2u,%2u)\n", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3]);
    return 0;
}
