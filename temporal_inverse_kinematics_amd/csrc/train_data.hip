// train_data.hip — the training-data generation of AmassDataset
// (mmskeleton/datasets/data_amass.py:87-218) on the GPU: SURVEY.md §8f row 4
// (the data half of the training path).
//
//  * rotate_root_z_kernel: regenerate_data's root-orientation augmentation
//    (data_amass.py:184-190): new_root = rotvec(R_z(angle) * R(root)), computed
//    in float64 the way scipy.spatial.transform.Rotation does it (from_rotvec /
//    quaternion product / as_rotvec with their small-angle series).
//  * train_windows_kernel: __getitem__ (data_amass.py:125-154) for a batch of
//    items, one workgroup per item: the edge-padded window of the FK joints
//    (sample_window :18-42), the SMPL-X -> COCO-17 gather (convert_smplx
//    :45-55), root-relative (:133-135), the per-joint Gaussian keypoint noise
//    (_aug_3d_keypoints :65-84: sigma_jc = mean-over-frames of the per-frame
//    bbox size_c x coco_sigma_j x 0.003, used as the VARIANCE of the diagonal
//    covariance), and the target pose row (the last frame of the pose window,
//    first 66 values). The reference draws the noise from numpy's global
//    generator; here it is a counter-based normal (splitmix64 + Box-Muller)
//    keyed by (seed, item, value), so any batch split gives the same values
//    (oracle/amass.py restates the generator).
#include <hip/hip_runtime.h>

#include "train_data.h"

namespace tik {

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// standard normal number n of the stream `key` (Box-Muller on two 53-bit uniforms)
__device__ __forceinline__ double counter_normal(unsigned long long key, unsigned long long n) {
    const unsigned long long a = splitmix64(key + 2 * n), b = splitmix64(key + 2 * n + 1);
    const double u1 = (double)((a >> 11) + 1) * 0x1.0p-53;   // (0, 1]
    const double u2 = (double)(b >> 11) * 0x1.0p-53;         // [0, 1)
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

__global__ void rotate_root_z_kernel(float* __restrict__ poses, int F, int ld, double angle) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= F) return;
    float* p = poses + (size_t)f * ld;
    const double vx = p[0], vy = p[1], vz = p[2];
    // scipy Rotation.from_rotvec: q = (scale v, cos(angle/2)), scale = sin(angle/2)/angle
    const double th = sqrt(vx * vx + vy * vy + vz * vz);
    const double th2 = th * th;
    const double sc = th <= 1e-3 ? 0.5 - th2 / 48.0 + th2 * th2 / 3840.0 : sin(0.5 * th) / th;
    const double qx = sc * vx, qy = sc * vy, qz = sc * vz, qw = cos(0.5 * th);
    // R_z(angle): (0, 0, sin(a/2), cos(a/2)); product p * q (scipy composition aug * org)
    const double pz = sin(0.5 * angle), pw = cos(0.5 * angle);
    double rx = pw * qx - pz * qy;
    double ry = pw * qy + pz * qx;
    double rz = pw * qz + pz * qw;
    double rw = pw * qw - pz * qz;
    // as_rotvec: canonical w >= 0, angle = 2 atan2(|xyz|, w), scale = angle / sin(angle/2)
    if (rw < 0.0) { rx = -rx; ry = -ry; rz = -rz; rw = -rw; }
    const double n = sqrt(rx * rx + ry * ry + rz * rz);
    const double a = 2.0 * atan2(n, rw);
    const double a2 = a * a;
    const double s = a <= 1e-3 ? 2.0 + a2 / 12.0 + 7.0 * a2 * a2 / 2880.0 : a / sin(0.5 * a);
    p[0] = (float)(s * rx);
    p[1] = (float)(s * ry);
    p[2] = (float)(s * rz);
}

// one workgroup per item; W = 2h+1 frames x 17 COCO joints in LDS
__global__ __launch_bounds__(256) void train_windows_kernel(TrainWinArgs a) {
    __shared__ float kp[TW_MAXW * 17 * 3];
    __shared__ float fsz[TW_MAXW * 3];   // per-frame bbox size
    __shared__ float msz[3];
    const int item = blockIdx.x, tid = threadIdx.x;
    const int W = 2 * a.h + 1;
    const int s0 = a.item_start[item], F = a.item_len[item], idx = a.item_idx[item];
    // window frames, edge-padded (sample_window), SMPL-X -> COCO gather
    for (int p = tid; p < W * 17; p += 256) {
        const int k = p / 17, j = p - 17 * k;
        int t = idx - a.h + k;
        t = t < 0 ? 0 : (t >= F ? F - 1 : t);
        const float* src = a.joints + ((size_t)(s0 + t) * a.n_joints + a.map[j]) * 3;
        kp[p * 3] = src[0];
        kp[p * 3 + 1] = src[1];
        kp[p * 3 + 2] = src[2];
    }
    __syncthreads();
    // root-relative: root = 0.5 (hip_l + hip_r) of the same frame (data_amass.py:133-135)
    __shared__ float root[TW_MAXW * 3];
    for (int q = tid; q < W * 3; q += 256) {
        const int k = q / 3, c = q - 3 * k;
        root[q] = a.relative ? 0.5f * (kp[(k * 17 + 11) * 3 + c] + kp[(k * 17 + 12) * 3 + c]) : 0.f;
    }
    __syncthreads();
    for (int p = tid; p < W * 17; p += 256) {
        const int k = p / 17;
#pragma unroll
        for (int c = 0; c < 3; ++c) kp[p * 3 + c] -= root[k * 3 + c];
    }
    __syncthreads();
    if (a.add_noise) {
        // per-frame bbox size (max - min over the 17 joints) ...
        for (int q = tid; q < W * 3; q += 256) {
            const int k = q / 3, c = q - 3 * k;
            float lo = kp[(k * 17) * 3 + c], hi = lo;
            for (int j = 1; j < 17; ++j) {
                const float v = kp[(k * 17 + j) * 3 + c];
                lo = fminf(lo, v);
                hi = fmaxf(hi, v);
            }
            fsz[q] = hi - lo;
        }
        __syncthreads();
        // ... averaged over the frames (float64 sum, as a float32 mean would be ordered differently anyway)
        if (tid < 3) {
            double s = 0.0;
            for (int k = 0; k < W; ++k) s += fsz[k * 3 + tid];
            msz[tid] = (float)(s / W);
        }
        __syncthreads();
        const unsigned long long key = splitmix64(a.seed ^ splitmix64((unsigned long long)a.item_uid[item]));
        for (int p = tid; p < W * 17; p += 256) {
            const int j = p % 17;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float var = msz[c] * a.sigma[j] * 0.003f;   // the covariance diagonal
                const double z = counter_normal(key, (unsigned long long)(p * 3 + c));
                kp[p * 3 + c] += (float)(sqrt((double)var) * z);
            }
        }
        __syncthreads();
    }
    float* o = a.windows + (size_t)item * W * 17 * 3;
    for (int i = tid; i < W * 17 * 3; i += 256) o[i] = kp[i];
    // target: the last frame of the pose window (edge-padded), first 66 values
    int tl = idx + a.h;
    tl = tl >= F ? F - 1 : tl;
    const float* ps = a.poses + (size_t)(s0 + tl) * a.pose_ld;
    for (int i = tid; i < 66; i += 256) a.target[(size_t)item * 66 + i] = ps[i];
}

hipError_t launch_rotate_root_z(float* poses, int F, int ld, double angle, hipStream_t st) {
    if (F <= 0) return hipSuccess;
    (void)hipGetLastError();
    hipLaunchKernelGGL(rotate_root_z_kernel, dim3((F + 255) / 256), dim3(256), 0, st, poses, F, ld, angle);
    return hipGetLastError();
}

hipError_t launch_train_windows(const TrainWinArgs& a, int B, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    if (2 * a.h + 1 > TW_MAXW) return hipErrorInvalidValue;
    (void)hipGetLastError();
    hipLaunchKernelGGL(train_windows_kernel, dim3(B), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace tik
