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
#include "dev_common.h"

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

// One wave per body (4 bodies per 256-thread workgroup), lane j = joint j:
// Rodrigues and the regressed joint of every joint in parallel, then the
// kinematic tree composed level by level (depth 0 .. maxdepth) through LDS,
// each joint's G_j from its parent's G_p written at the previous level. The
// per-element arithmetic is the sequential smplx recursion's, unchanged.
constexpr int FKW = 4;   // bodies (waves) per workgroup

__global__ __launch_bounds__(64 * FKW) void fk_chain_kernel(FkChainArgs a) {
    __shared__ float sG[FKW][55 * 12];
    __shared__ float sJ[FKW][55 * 3];
    __shared__ float sR[FKW][55 * 9];
    __shared__ float sF[FKW][512];
    const int wv = threadIdx.x >> 6, j = threadIdx.x & 63;
    const int b = blockIdx.x * FKW + wv;
    const bool live = b < a.B;
    const int NS = a.nb + a.ne;
    const int bb = live ? b : 0;
    float shp[32];
#pragma unroll
    for (int l = 0; l < 32; ++l) {
        float v = 0.f;
        if (l < NS) {
            if (l < a.nb) v = a.betas ? a.betas[(size_t)bb * a.nb + l] : 0.f;
            else v = a.expr ? a.expr[(size_t)bb * a.ne + (l - a.nb)] : 0.f;
        }
        shp[l] = v;
    }
    const float* pose = a.pose + (size_t)bb * 55 * 3;
    float* F = sF[wv];
    // (1) per joint: R_j, J_j, the pose feature vec(R_j - I)
    float R[9], J[3];
    int dj = -1;
    if (j < 55) {
        rodrigues_smplx(pose[j * 3] + a.pose_mean[j * 3], pose[j * 3 + 1] + a.pose_mean[j * 3 + 1],
                        pose[j * 3 + 2] + a.pose_mean[j * 3 + 2], R);
        for (int c = 0; c < 3; ++c) {
            float v = a.jt[j * 3 + c];
            const float* d = a.jd + ((size_t)j * 3 + c) * NS;
            for (int l = 0; l < NS; ++l) v = fmaf(d[l], shp[l], v);
            J[c] = v;
        }
        for (int k = 0; k < 9; ++k) sR[wv][j * 9 + k] = R[k];
        for (int c = 0; c < 3; ++c) sJ[wv][j * 3 + c] = J[c];
        if (j > 0)
            for (int k = 0; k < 9; ++k) F[9 * (j - 1) + k] = R[k] - ((k % 4) == 0 ? 1.f : 0.f);
        dj = a.depth[j];
    }
    // feature tail: [betas | expression | 1 | 0 ...]
    for (int k = 486 + j; k < a.kp; k += 64) {
        const int l = k - 486;
        F[k] = l < NS ? shp[l] : (l == NS ? 1.0f : 0.f);
    }
    __syncthreads();
    // (2) the kinematic chain, one tree level at a time
    float g[12];
    for (int d = 0; d <= a.maxdepth; ++d) {
        if (dj == d) {
            const int p = a.parents[j];
            if (p < 0) {
                for (int r = 0; r < 3; ++r) {
                    g[4 * r] = R[3 * r]; g[4 * r + 1] = R[3 * r + 1]; g[4 * r + 2] = R[3 * r + 2]; g[4 * r + 3] = J[r];
                }
            } else {
                float P[12];
                for (int e = 0; e < 12; ++e) P[e] = sG[wv][p * 12 + e];
                const float t0 = J[0] - sJ[wv][p * 3], t1 = J[1] - sJ[wv][p * 3 + 1], t2 = J[2] - sJ[wv][p * 3 + 2];
                for (int r = 0; r < 3; ++r) {
                    for (int c = 0; c < 3; ++c)
                        g[4 * r + c] = P[4 * r] * R[c] + P[4 * r + 1] * R[3 + c] + P[4 * r + 2] * R[6 + c];
                    g[4 * r + 3] = P[4 * r] * t0 + P[4 * r + 1] * t1 + P[4 * r + 2] * t2 + P[4 * r + 3];
                }
            }
            for (int e = 0; e < 12; ++e) sG[wv][j * 12 + e] = g[e];
        }
        __syncthreads();
    }
    const float tx = (live && a.transl) ? a.transl[bb * 3] : 0.f;
    const float ty = (live && a.transl) ? a.transl[bb * 3 + 1] : 0.f;
    const float tz = (live && a.transl) ? a.transl[bb * 3 + 2] : 0.f;
    // (3) joints, and A_j = G_j with translation t - R_G J_j (rows 12..15, joints 55.. zero)
    float A[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) A[e] = 0.f;
    if (j < 55) {
        float* jo = a.joints + (size_t)bb * a.njoints * 3;
        if (live) {
            jo[j * 3] = g[3] + tx;
            jo[j * 3 + 1] = g[7] + ty;
            jo[j * 3 + 2] = g[11] + tz;
        }
#pragma unroll
        for (int e = 0; e < 12; ++e) A[e] = g[e];
        for (int r = 0; r < 3; ++r)
            A[4 * r + 3] = g[4 * r + 3] - (g[4 * r] * J[0] + g[4 * r + 1] * J[1] + g[4 * r + 2] * J[2]);
    }
    // the neck-chain product in the reference's order: rel = R[c_{n-1}] ... R[c_1] R[c_0]
    if (j == 0 && live && a.dyn_bin) {
        float rel[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        for (int k = 0; k < a.nchain; ++k) {
            const float* Rk = sR[wv] + a.chain[k] * 9;
            float nr[9];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c)
                    nr[3 * r + c] = Rk[3 * r] * rel[c] + Rk[3 * r + 1] * rel[3 + c] + Rk[3 * r + 2] * rel[6 + c];
            for (int e = 0; e < 9; ++e) rel[e] = nr[e];
        }
        const float sy = sqrtf(rel[0] * rel[0] + rel[3] * rel[3]);
        const float eul = atan2f(-rel[6], sy);
        float yd = -eul * 180.0f / 3.14159265358979323846f;
        yd = fminf(yd, 39.0f);
        int y = (int)rintf(yd);
        const int neg = y < 0, mask = y < -39;
        const int negv = mask ? 78 : 39 - y;
        a.dyn_bin[b] = neg ? negv : y;
    }
    if (!live) return;   // no barrier below
    // (4) outputs: lane j holds column j of A (kj = 64 columns)
    if (a.ablk) {
        const int ar = a.arows == 12 ? 12 : 16;
        float* G = a.ablk + (size_t)b * ar * a.kj;
        for (int e = 0; e < ar; ++e)
            if (j < a.kj) G[e * a.kj + j] = A[e];
    }
    if (a.ajt && j < 55) {   // joint-major [55][B][12]: lane j writes its 12 entries
        f32x4* o = reinterpret_cast<f32x4*>(a.ajt + ((size_t)j * a.B + b) * 12);
        o[0] = f32x4{A[0], A[1], A[2], A[3]};
        o[1] = f32x4{A[4], A[5], A[6], A[7]};
        o[2] = f32x4{A[8], A[9], A[10], A[11]};
    }
    if (a.feat) {
        float* f = a.feat + (size_t)b * a.kp;
        for (int k = j; k < a.kp; k += 64) f[k] = F[k];
    }
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

// Sparse skinning. A workgroup owns 256 consecutive vertices (thread = vertex,
// its nz {joint, weight} pairs in registers) and walks a run of body tiles of
// SBT = 4 bodies: the tile's A_j (SBT x 55 x 12 floats) sits in LDS, double
// buffered — the next tile's A_j and v_posed rows are loaded into registers
// during the current tile's math, written to the other buffer after it, one
// barrier per tile. Loads and stores are 12 B per thread, consecutive across
// lanes (vertex-major rows), so every wave moves 768 contiguous bytes.
namespace fksp {
constexpr int AB = 55 * 12;                     // floats of A_j per body
}  // namespace fksp

template <int NZ, int SBT>
__global__ __launch_bounds__(256) void fk_skin_sparse_kernel(FkSkinSpArgs a, int runs) {
    using namespace fksp;
    constexpr int ABUF = SBT * AB;                  // floats per buffer (SBT = 4: 10,560 B)
    constexpr int NA4 = (ABUF / 4 + 255) / 256;     // f32x4 loads per thread per tile
    __shared__ __attribute__((aligned(16))) float sA[2][ABUF];
    const int tid = threadIdx.x;
    const int v = blockIdx.x * 256 + tid;
    const bool vok = v < a.V;
    const int vc = vok ? v : a.V - 1;
    const int nbt = (a.B + SBT - 1) / SBT;
    const int t0 = (int)((long long)blockIdx.y * nbt / runs), t1 = (int)((long long)(blockIdx.y + 1) * nbt / runs);
    if (t0 >= t1) return;
    int jo[NZ];
    float wv[NZ];
#pragma unroll
    for (int k = 0; k < NZ; ++k) {
        const int2 e = a.nzw[(size_t)vc * NZ + k];
        jo[k] = e.x * 12;
        wv[k] = __builtin_bit_cast(float, e.y);
    }
    f32x4 pa[NA4];
    auto load = [&](int t, float (&pv)[SBT][3]) __attribute__((always_inline)) {   // tile t's A_j and v_posed into registers
        // A_j is joint-major in memory ([55][B][12]): slot q = (body, joint, quarter) of the
        // tile's body-major LDS image reads joint j's 16 B of body t SBT + body
        const int nb = min(SBT, a.B - t * SBT);
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
            const int q = tid + 256 * i;
            const int bb = q / (AB / 4), r = q - bb * (AB / 4), jj = r / 3;
            pa[i] = q < nb * (AB / 4)
                        ? *reinterpret_cast<const f32x4*>(a.ajt + ((size_t)jj * a.ajt_ld + t * SBT + bb) * 12 + 4 * (r - 3 * jj))
                        : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int b = 0; b < SBT; ++b) {
            const int body = min(t * SBT + b, a.B - 1);
            // streaming (nt) loads: v_posed is read once
            const float* q = a.vposed + (size_t)body * a.ldv + 3 * vc;
            pv[b][0] = __builtin_nontemporal_load(q);
            pv[b][1] = __builtin_nontemporal_load(q + 1);
            pv[b][2] = __builtin_nontemporal_load(q + 2);
        }
    };
    auto put = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
            const int q = tid + 256 * i;
            if (q < ABUF / 4) reinterpret_cast<f32x4*>(sA[buf])[q] = pa[i];
        }
    };
    auto tile = [&](int t, const float (&cv)[SBT][3], float (&nv)[SBT][3]) __attribute__((always_inline)) {
        if (t + 1 < t1) load(t + 1, nv);
        const float* A = sA[t & 1];
#pragma unroll
        for (int b = 0; b < SBT; ++b) {
            const int body = t * SBT + b;
            const int bc = body < a.B ? body : a.B - 1;
            float T[12];
#pragma unroll
            for (int e = 0; e < 12; ++e) T[e] = 0.f;
#pragma unroll
            for (int k = 0; k < NZ; ++k) {
                const f32x4* r = reinterpret_cast<const f32x4*>(A + b * AB + jo[k]);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const f32x4 x = r[q];
#pragma unroll
                    for (int e = 0; e < 4; ++e) T[4 * q + e] = fmaf(wv[k], x[e], T[4 * q + e]);
                }
                if (k % 4 == 3) __builtin_amdgcn_sched_barrier(0);   // at most four joints' reads in flight
            }
            float o[3];
#pragma unroll
            for (int g = 0; g < 3; ++g)
                o[g] = fmaf(T[4 * g], cv[b][0], fmaf(T[4 * g + 1], cv[b][1], fmaf(T[4 * g + 2], cv[b][2], T[4 * g + 3]))) +
                       a.transl[bc * 3 + g];
            if (vok && body < a.B) {   // streaming (nt) stores: -4 % skinning (profiles/r06_ab_fk_nontemporal.txt)
                float* d = a.verts + (size_t)body * 3 * a.V + 3 * v;
                __builtin_nontemporal_store(o[0], d);
                __builtin_nontemporal_store(o[1], d + 1);
                __builtin_nontemporal_store(o[2], d + 2);
            }
            __builtin_amdgcn_sched_barrier(0);   // one body's LDS reads in flight at a time (registers)
        }
        if (t + 1 < t1) put((t + 1) & 1);
        __syncthreads();
    };
    float va[SBT][3], vb[SBT][3];
    load(t0, va);
    put(t0 & 1);   // tile t reads buffer t & 1
    __syncthreads();
    for (int t = t0; t < t1; t += 2) {   // unrolled by two: the v_posed buffers swap statically
        tile(t, va, vb);
        if (t + 1 < t1) tile(t + 1, vb, va);
    }
}

hipError_t launch_fk_skin_sparse(const FkSkinSpArgs& a, hipStream_t st) {
    if (a.B <= 0 || a.V <= 0) return hipSuccess;
    if ((a.nz != 4 && a.nz != 8 && a.nz != 16) || !a.ajt || !a.nzw || !a.vposed || !a.verts || !a.transl || a.ldv < 3 * a.V ||
        a.ajt_ld < a.B)
        return hipErrorInvalidValue;
    constexpr int sbt = 4;   // bodies per tile (8: same time, more VGPRs)
    const int vt = (a.V + 255) / 256, nbt = (a.B + sbt - 1) / sbt;
    // about 16 workgroups per CU (3 resident at 134 VGPRs), each walking a run of body tiles:
    // shorter runs than 4 per CU balance better (profiles/r06_ab_fk_landmarks_wpc.txt: -1 %)
    int runs = (16 * (a.ncu > 0 ? a.ncu : 256) + vt - 1) / vt;
    runs = runs < nbt ? runs : nbt;
    (void)hipGetLastError();
    const dim3 grid(vt, runs);
    if (a.nz == 4) hipLaunchKernelGGL((fk_skin_sparse_kernel<4, sbt>), grid, dim3(256), 0, st, a, runs);
    else if (a.nz == 8) hipLaunchKernelGGL((fk_skin_sparse_kernel<8, sbt>), grid, dim3(256), 0, st, a, runs);
    else hipLaunchKernelGGL((fk_skin_sparse_kernel<16, sbt>), grid, dim3(256), 0, st, a, runs);
    return hipGetLastError();
}

hipError_t launch_fk_chain(const FkChainArgs& a, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    (void)hipGetLastError();
    if (a.kj != 64 || a.kp % 32 || a.kp > 512 || !a.depth) return hipErrorInvalidValue;
    hipLaunchKernelGGL(fk_chain_kernel, dim3((a.B + FKW - 1) / FKW), dim3(64 * FKW), 0, st, a);
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
