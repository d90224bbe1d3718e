// Standalone launch test of libtik.so (no torch): aa->rotmat on 4 vectors.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../include/tik.h"
int main() {
    float h[12] = {0, 0, 0, 0.1f, 0.2f, 0.3f, 1, 0, 0, 0, 0, 3.0f};
    float *d, *R;
    hipMalloc(&d, sizeof(h)); hipMalloc(&R, 36 * sizeof(float));
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    int rc = tik_aa_to_rotmat(d, 4, R, nullptr);
    printf("rc=%d err=%s\n", rc, tik_last_error());
    float out[36];
    hipMemcpy(out, R, sizeof(out), hipMemcpyDeviceToHost);
    printf("R[3]: %f %f %f / %f %f %f\n", out[9], out[10], out[11], out[12], out[13], out[14]);
    return rc;
}
