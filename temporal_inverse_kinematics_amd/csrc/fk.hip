// fk.hip — SMPL-X forward kinematics around the two LBS GEMMs
// (the FK check of common/smpl_util.py:22-82 -> third-party smplx.SMPLX.forward).
//
//   fk_chain_kernel      one thread per body: smplx batch_rodrigues for the 55
//                        joints, regressed joints J = J_template + J_dirs.shape
//                        (J_regressor folded into the blend shapes on the host),
//                        the kinematic chain G_j = G_parent [R_j | J_j - J_parent],
//                        A_j = G_j - [0 | G_j J_j], the 486-d pose feature
//                        vec(R_j - I), the dynamic face-contour bin.
//   fk_landmark_kernel   the 21 vertex-picked joints, 51 barycentric face
//                        landmarks and 17 dynamic contour landmarks.
// The two GEMMs (pose/shape blend shapes; skinning + vertex transform) run on
// the fp32-MFMA implicit-GEMM kernel (cgemm.hip, CFG_T128x128 / CFG_S128x128).
#include "fk.h"

namespace tik {

__device__ inline void rodrigues_smplx(float x, float y, float z, float R[9]) {
    // smplx lbs.batch_rodrigues: angle = ||v + 1e-8||, rot_dir = v / angle,
    // R = I + sin K + (1 - cos) K K
    const float ax = x + 1e-8f, ay = y + 1e-8f, az = z + 1e-8f;
    const float ang = sqrtf(ax * ax + ay * ay + az * az);
    const float inv = 1.0f / ang;
    const float dx = x * inv, dy = y * inv, dz = z * inv;
    float s, c;
    sincosf(ang, &s, &c);
    const float oc = 1.0f - c;
    const float d2 = dx * dx + dy * dy + dz * dz;
    // K = [0,-dz,dy; dz,0,-dx; -dy,dx,0];  (K K)_ij = d_i d_j - delta_ij |d|^2
    R[0] = 1.f + oc * (dx * dx - d2);  R[1] = -s * dz + oc * dx * dy;      R[2] = s * dy + oc * dx * dz;
    R[3] = s * dz + oc * dx * dy;      R[4] = 1.f + oc * (dy * dy - d2);  R[5] = -s * dx + oc * dy * dz;
    R[6] = -s * dy + oc * dx * dz;     R[7] = s * dx + oc * dy * dz;      R[8] = 1.f + oc * (dz * dz - d2);
}

__global__ void fk_chain_kernel(FkChainArgs a) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.B) return;
    const int NS = a.nb + a.ne;
    float shp[32];
    for (int l = 0; l < NS && l < 32; ++l) {
        float v = 0.f;
        if (l < a.nb) v = a.betas ? a.betas[(size_t)b * a.nb + l] : 0.f;
        else v = a.expr ? a.expr[(size_t)b * a.ne + (l - a.nb)] : 0.f;
        shp[l] = v;
    }
    float* feat = a.feat + (size_t)b * a.kp;
    float* G = a.ablk + (size_t)b * 16 * a.kj;        // [16][kj], column j = joint
    const float* pose = a.pose + (size_t)b * 55 * 3;
    const float tx = a.transl ? a.transl[b * 3] : 0.f;
    const float ty = a.transl ? a.transl[b * 3 + 1] : 0.f;
    const float tz = a.transl ? a.transl[b * 3 + 2] : 0.f;
    float* jo = a.joints + (size_t)b * a.njoints * 3;

    auto Jpos = [&](int j, float J[3]) {
        for (int c = 0; c < 3; ++c) {
            float v = a.jt[j * 3 + c];
            const float* d = a.jd + ((size_t)j * 3 + c) * NS;
            for (int l = 0; l < NS; ++l) v = fmaf(d[l], shp[l], v);
            J[c] = v;
        }
    };
    float rel[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};   // neck-chain rotation product
    for (int j = 0; j < 55; ++j) {
        float R[9], J[3];
        rodrigues_smplx(pose[j * 3] + a.pose_mean[j * 3], pose[j * 3 + 1] + a.pose_mean[j * 3 + 1],
                        pose[j * 3 + 2] + a.pose_mean[j * 3 + 2], R);
        if (j > 0)
            for (int k = 0; k < 9; ++k) feat[9 * (j - 1) + k] = R[k] - ((k % 4) == 0 ? 1.f : 0.f);
        Jpos(j, J);
        float g[12];
        const int p = a.parents[j];
        if (p < 0) {
            for (int r = 0; r < 3; ++r) {
                g[4 * r] = R[3 * r]; g[4 * r + 1] = R[3 * r + 1]; g[4 * r + 2] = R[3 * r + 2]; g[4 * r + 3] = J[r];
            }
        } else {
            float Jp[3], P[12];
            Jpos(p, Jp);
            for (int e = 0; e < 12; ++e) P[e] = G[e * a.kj + p];
            const float t0 = J[0] - Jp[0], t1 = J[1] - Jp[1], t2 = J[2] - Jp[2];
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c)
                    g[4 * r + c] = P[4 * r] * R[c] + P[4 * r + 1] * R[3 + c] + P[4 * r + 2] * R[6 + c];
                g[4 * r + 3] = P[4 * r] * t0 + P[4 * r + 1] * t1 + P[4 * r + 2] * t2 + P[4 * r + 3];
            }
        }
        for (int e = 0; e < 12; ++e) G[e * a.kj + j] = g[e];
        jo[j * 3] = g[3] + tx;
        jo[j * 3 + 1] = g[7] + ty;
        jo[j * 3 + 2] = g[11] + tz;
    }
    // the neck-chain product in the reference's order: rel = R[c_{n-1}] ... R[c_1] R[c_0]
    for (int k = 0; k < a.nchain; ++k) {
        const int j = a.chain[k];
        float R[9], nr[9];
        rodrigues_smplx(pose[j * 3] + a.pose_mean[j * 3], pose[j * 3 + 1] + a.pose_mean[j * 3 + 1],
                        pose[j * 3 + 2] + a.pose_mean[j * 3 + 2], R);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                nr[3 * r + c] = R[3 * r] * rel[c] + R[3 * r + 1] * rel[3 + c] + R[3 * r + 2] * rel[6 + c];
        for (int e = 0; e < 9; ++e) rel[e] = nr[e];
    }
    if (a.dyn_bin) {
        const float sy = sqrtf(rel[0] * rel[0] + rel[3] * rel[3]);
        const float eul = atan2f(-rel[6], sy);
        float yd = -eul * 180.0f / 3.14159265358979323846f;
        yd = fminf(yd, 39.0f);
        int y = (int)rintf(yd);
        const int neg = y < 0, mask = y < -39;
        const int negv = mask ? 78 : 39 - y;
        a.dyn_bin[b] = neg ? negv : y;
    }
    // A_j = G_j with translation t - R_G J_j; pad rows 12..15 and joints 55..kj-1 with zeros
    for (int j = 0; j < 55; ++j) {
        float J[3];
        Jpos(j, J);
        float g[12];
        for (int e = 0; e < 12; ++e) g[e] = G[e * a.kj + j];
        for (int r = 0; r < 3; ++r)
            G[(4 * r + 3) * a.kj + j] = g[4 * r + 3] - (g[4 * r] * J[0] + g[4 * r + 1] * J[1] + g[4 * r + 2] * J[2]);
    }
    for (int e = 0; e < 16; ++e)
        for (int j = (e < 12 ? 55 : 0); j < a.kj; ++j) G[e * a.kj + j] = 0.f;
    // feature tail: [betas | expression | 1 | 0 ...]
    const int nf = 54 * 9;
    for (int l = 0; l < NS; ++l) feat[nf + l] = shp[l];
    feat[nf + NS] = 1.0f;
    for (int k = nf + NS + 1; k < a.kp; ++k) feat[k] = 0.f;
}

__global__ void fk_landmark_kernel(FkLmkArgs a) {
    const int per = a.nextra + a.nlmk + a.ndyn;
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= (long long)a.B * per) return;
    const int b = (int)(p / per);
    const int k = (int)(p - (long long)b * per);
    const float* vb = a.verts + (size_t)b * a.V * 3;
    float o[3];
    if (k < a.nextra) {
        const int v = a.extra[k];
        o[0] = vb[3 * v]; o[1] = vb[3 * v + 1]; o[2] = vb[3 * v + 2];
    } else {
        int f;
        const float* bc;
        if (k < a.nextra + a.nlmk) {
            const int l = k - a.nextra;
            f = a.lmk_faces[l];
            bc = a.lmk_bary + 3 * l;
        } else {
            const int d = k - a.nextra - a.nlmk;
            const int bin = a.dyn_bin[b];
            f = a.dyn_faces[bin * a.ndyn + d];
            bc = a.dyn_bary + ((size_t)bin * a.ndyn + d) * 3;
        }
        const float sb = bc[0] + bc[1] + bc[2];
        for (int c = 0; c < 3; ++c) {
            float s = 0.f;
            for (int i = 0; i < 3; ++i) s = fmaf(bc[i], vb[3 * a.faces[3 * f + i] + c], s);
            // vertices carry transl; landmarks are taken before it, then transl is added
            const float t = a.transl ? a.transl[b * 3 + c] : 0.f;
            o[c] = s + t * (1.0f - sb);
        }
    }
    float* jo = a.joints + ((size_t)b * a.njoints + 55 + k) * 3;
    jo[0] = o[0]; jo[1] = o[1]; jo[2] = o[2];
}

hipError_t launch_fk_chain(const FkChainArgs& a, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    (void)hipGetLastError();
    hipLaunchKernelGGL(fk_chain_kernel, dim3((a.B + 63) / 64), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_fk_landmarks(const FkLmkArgs& a, hipStream_t st) {
    const long long n = (long long)a.B * (a.nextra + a.nlmk + a.ndyn);
    if (n <= 0) return hipSuccess;
    (void)hipGetLastError();
    hipLaunchKernelGGL(fk_landmark_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace tik
