#pragma once
#include <hip/hip_runtime.h>

namespace tik {

hipError_t launch_data_bn(const float* x, int n_px, int V, int C, const float* scale,
                          const float* shift, float* xb, hipStream_t st);
hipError_t launch_aa_to_rotmat(const float* aa, int n, float* R, hipStream_t st);
hipError_t launch_window_gather(const float* seq, int F, int V, int idx0, int n_idx, int h, int ra,
                                int rb, int relative, float* out, hipStream_t st);
hipError_t launch_gconv(const float* x, int N, int Cin, int T, int V, const float* A, int K,
                        const float* W, const float* b, int Cout, int tk, int ts, int tp, int td,
                        int To, float* out, hipStream_t st);

// moveai_3d -> COCO-17 (inference.py:121-133): gather by map (17 entries, -1 = none),
// COCO 0 = mid of the last two joints (the ears), 1 / 2 = the last-but-one / last
// joint, then (x, y, z) -> (x, z, -y). joints (F,J,3) -> out (F,17,3)
hipError_t launch_moveai_to_coco(const float* joints, int F, int J, const int* map17, float* out, hipStream_t st);

hipError_t launch_pad_channels(const float* x, long long rows, int C, int Cp, float* y, hipStream_t st);

hipError_t launch_stream_push(float* ring, int W, int nv, int* count, const float* frame, hipStream_t st);
hipError_t launch_stream_window(const float* ring, int W, int V, const int* count, int h, int ra, int rb,
                                int relative, float* out, hipStream_t st);

// debug: order-independent checksum (sum of 32-bit words, index-weighted) of a buffer into *out
hipError_t launch_checksum(const void* p, size_t bytes, unsigned long long* out, hipStream_t st);

}  // namespace tik
