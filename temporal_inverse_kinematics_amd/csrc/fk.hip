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
#include "cgemm3_dev.h"

namespace tik {

typedef f16x8 f16x8s;

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

__device__ __forceinline__ unsigned short f16bits(float x) { return __builtin_bit_cast(unsigned short, (_Float16)x); }

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
    if (a.ajt && j < 55) {   // joint-major: lane j writes its 12 entries
        f32x4* o = reinterpret_cast<f32x4*>(a.ajt + ((size_t)b * 55 + j) * 12);
        o[0] = f32x4{A[0], A[1], A[2], A[3]};
        o[1] = f32x4{A[4], A[5], A[6], A[7]};
        o[2] = f32x4{A[8], A[9], A[10], A[11]};
    }
    if (a.ablk_sb) {   // rows b*16+e, K = joint: block j/32, hi at j%32, lo 32 further
        unsigned short* G = a.ablk_sb + (size_t)b * 16 * (2 * a.kj);
        for (int e = 0; e < 16; ++e) {
            const float x = A[e];
            const _Float16 h = (_Float16)x;
            const _Float16 l = (_Float16)(x - (float)h);
            unsigned short* row = G + (size_t)e * 2 * a.kj + (j >> 5) * 64 + (j & 31);
            row[0] = __builtin_bit_cast(unsigned short, h);
            row[32] = __builtin_bit_cast(unsigned short, l);
        }
    }
    if (a.feat) {
        float* f = a.feat + (size_t)b * a.kp;
        for (int k = j; k < a.kp; k += 64) f[k] = F[k];
    }
    if (a.feat_sb) {   // kp/32 blocks of [hi x32 | lo x32]: lane j writes 8 channels of block j/4
        unsigned short* f = a.feat_sb + (size_t)b * 2 * a.kp;
        for (int q = j; q < a.kp / 8; q += 64) {
            const int blk = q >> 2, c0 = (q & 3) * 8;
            f16x8s hv, lv;
            for (int e = 0; e < 8; ++e) {
                const float x = F[blk * 32 + c0 + e];
                const _Float16 h = (_Float16)x;
                hv[e] = h;
                lv[e] = (_Float16)(x - (float)h);
            }
            *reinterpret_cast<f16x8s*>(f + blk * 64 + c0) = hv;
            *reinterpret_cast<f16x8s*>(f + blk * 64 + 32 + c0) = lv;
        }
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

// Skinning + vertex transform. A workgroup owns 128 vertices (their skinning
// weights W stay in LDS) and walks a run of body tiles of 8 bodies = 128 rows
// b*16+e of A (K = 64 joints, 2 split blocks): the next tile's A is DMA'd into
// the other half of a double buffer and the tile's v_posed rows are loaded
// into registers before the MFMAs (f16x3, cgemm3's a_lo b_hi + a_hi b_lo +
// a_hi b_hi). The epilogue works on the accumulators directly: one 16-row
// fragment is one body, lane group g < 3 holds row g of T_v(b) for vertex
// lane&15, i.e. output coordinate g, in the order of smplx lbs:
// T[g,:3] v_posed + T[g,3], then + transl. Every wave issues a fixed number of
// vector-memory instructions per tile (rows past the batch are clamped on
// load and redirected to a trash line on store), so the vmcnt waits are exact.
namespace fks {
constexpr int BR = 128, BV = 128, IMG = 128 * 128;   // rows (8 bodies x 16), vertices, one block image
constexpr int NW = 8;                                // waves: 2 (rows) x 4 (vertex columns)
constexpr int FM = 4, FN = 2;                        // 16x16 fragments per wave
constexpr int NDA = 2 * 16 / NW;                     // DMA instructions per wave per operand (2 block images x 16)
constexpr int NLD = FM * FN + FM;                    // loads per wave per tile: v_posed (one dwordx3 per vertex) + transl
constexpr int NST = FM * FN;                         // vertex stores per wave per tile
constexpr int SMEM = 2 * IMG + 2 * 2 * IMG;          // W (2 blocks) + A double buffer (2 x 2 blocks): 96 KB
}  // namespace fks

__global__ __launch_bounds__(512, 1) void fk_skin_kernel(FkSkinArgs a, int runs) {
    using namespace fks;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int v0 = blockIdx.x * BV;
    const int nbt = (a.B + 7) / 8;   // body tiles
    const int t0 = (int)((long long)blockIdx.y * nbt / runs), t1 = (int)((long long)(blockIdx.y + 1) * nbt / runs);
    const int M = a.B * 16;
    const i32x4 rA = buf_rsrc(a.ablk_sb, (unsigned)((long long)M * 256));
    const i32x4 rW = buf_rsrc(a.w_sb, (unsigned)((long long)a.V * 256));
    static_assert(NDA * NW == 2 * 16, "each operand is 2 block images of 16 DMA instructions");
    auto dma_img = [&](i32x4 r, int row0, int lim, int blk, unsigned char* img, int rg) {
        const int rr = rg * 8 + (lane >> 3), ck = (lane & 7) ^ sbf(rr), row = row0 + rr;
        const unsigned off = row < lim ? (unsigned)((row * 128 + blk * 64 + 8 * ck) * 2) : DMA_OOB;
        dma16(r, img + rg * 1024, off, 0);
    };
    auto issue_a = [&](int t) {   // 2 block images x 16 instructions over 8 waves; t >= t1: zero fill
        unsigned char* base = smem + 2 * IMG + (t & 1) * 2 * IMG;
#pragma unroll
        for (int j = 0; j < NDA; ++j) {
            const int idx = wave * NDA + j, blk = idx >> 4, rg = idx & 15;
            dma_img(rA, t * BR, t < t1 ? M : 0, blk, base + blk * IMG, rg);
        }
    };
    // W of this vertex tile, once; then the first A tile
#pragma unroll
    for (int j = 0; j < NDA; ++j) {
        const int idx = wave * NDA + j, blk = idx >> 4, rg = idx & 15;
        dma_img(rW, v0, a.V, blk, smem + blk * IMG, rg);
    }
    const int wm = wave >> 2, wn = wave & 3, g = lane >> 4, l15 = lane & 15;
    const int gc = g < 3 ? g : 2;   // lane group 3 carries no output row: mirrors row 2, stores to trash
    float* trash = reinterpret_cast<float*>(a.trash) + (tid & 255);
    // v_posed rows and translation entries of tile t (rows clamped into the batch): issued one
    // whole tile ahead, and before that tile's A DMA, so the wait for A(t) also retires them
    auto load_vp = [&](int t, float (&vp)[FM][FN][3], float (&tb)[FM]) {
#pragma unroll
        for (int i = 0; i < FM; ++i) tb[i] = a.transl[min(t * 8 + wm * FM + i, a.B - 1) * 3 + gc];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int body = min(t * 8 + wm * FM + i, a.B - 1);
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int v = min(v0 + wn * 32 + j * 16 + l15, a.V - 1);
                const float* p = a.vposed + (size_t)body * a.ldv + 3 * v;
                vp[i][j][0] = p[0]; vp[i][j][1] = p[1]; vp[i][j][2] = p[2];
            }
        }
    };
    int prev_st = 0;
    auto step = [&](int t, const float (&vp)[FM][FN][3], const float (&tb)[FM], float (&vpn)[FM][FN][3],
                    float (&tbn)[FM]) {
        load_vp(t + 1, vpn, tbn);
        issue_a(t + 1);
        // A(t) landed, and with it the older v_posed loads of tile t (younger: the last
        // tile's stores, tile t+1's loads and A DMA)
        wait_vm_dyn(prev_st + NLD + NDA);
        lds_barrier();   // not __syncthreads(): its fence would drain the prefetch (vmcnt(0))
        const unsigned char* Ab = smem + 2 * IMG + (t & 1) * 2 * IMG;
        f32x4 acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const unsigned char* A = Ab + kb * IMG;
            const unsigned char* Wb = smem + kb * IMG;
            f16x8 bh[FN], bl[FN];
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int r = wn * 32 + j * 16 + l15;
                bh[j] = *reinterpret_cast<const f16x8*>(Wb + sbo(r, g));
                bl[j] = *reinterpret_cast<const f16x8*>(Wb + sbo(r, 4 + g));
            }
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int r = wm * 64 + i * 16 + l15;
                const f16x8 ah = *reinterpret_cast<const f16x8*>(A + sbo(r, g));
                const f16x8 al = *reinterpret_cast<const f16x8*>(A + sbo(r, 4 + g));
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[j], acc[i][j], 0, 0, 0);
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every wave is done with A(t): its slot takes A(t+2) next tile
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int body = t * 8 + wm * FM + i;
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int v = v0 + wn * 32 + j * 16 + l15;
                const f32x4 T = acc[i][j];
                const float x = fmaf(T[0], vp[i][j][0], fmaf(T[1], vp[i][j][1], fmaf(T[2], vp[i][j][2], T[3])));
                const bool ok = g < 3 && body < a.B && v < a.V;
                float* o = ok ? a.verts + (size_t)body * 3 * a.V + 3 * v + g : trash;
                *o = x + tb[i];
            }
        }
        prev_st = NST;
    };
    float vpA[FM][FN][3], tbA[FM], vpB[FM][FN][3], tbB[FM];
    load_vp(t0, vpA, tbA);
    issue_a(t0);
    for (int t = t0; t < t1; t += 2) {   // unrolled by two: the prefetch buffers swap statically
        step(t, vpA, tbA, vpB, tbB);
        if (t + 1 < t1) step(t + 1, vpB, tbB, vpA, tbA);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

hipError_t launch_fk_skin(const FkSkinArgs& a, hipStream_t st) {
    if (a.B <= 0 || a.V <= 0) return hipSuccess;
    if (a.kj != 64 || !a.ablk_sb || !a.w_sb || !a.vposed || !a.verts || !a.trash || !a.transl || a.ldv < 3 * a.V ||
        (long long)a.B * 16 * 256 >= (1LL << 31) || (long long)a.B * a.ldv >= (1LL << 31))
        return hipErrorInvalidValue;
    const int vt = (a.V + fks::BV - 1) / fks::BV, nbt = (a.B + 7) / 8;
    // one workgroup per CU (96 KB of LDS) in all, each walking a run of body tiles
    int runs = 256 / vt > 1 ? 256 / vt : 1;
    runs = runs < nbt ? runs : nbt;
    (void)hipGetLastError();
    hipLaunchKernelGGL(fk_skin_kernel, dim3(vt, runs), dim3(512), 0, st, a, runs);
    return hipGetLastError();
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
        const f32x4* src = reinterpret_cast<const f32x4*>(a.ajt + (size_t)t * ABUF);
        const int nb = min(SBT, a.B - t * SBT);
#pragma unroll
        for (int i = 0; i < NA4; ++i) {
            const int q = tid + 256 * i;
            pa[i] = q < nb * (AB / 4) ? src[q] : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int b = 0; b < SBT; ++b) {
            const int body = min(t * SBT + b, a.B - 1);
            __builtin_memcpy(&pv[b][0], a.vposed + (size_t)body * a.ldv + 3 * vc, 12);
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
            if (vok && body < a.B) __builtin_memcpy(a.verts + (size_t)body * 3 * a.V + 3 * v, o, 12);
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
    if ((a.nz != 4 && a.nz != 8 && a.nz != 16) || !a.ajt || !a.nzw || !a.vposed || !a.verts || !a.transl || a.ldv < 3 * a.V)
        return hipErrorInvalidValue;
    constexpr int sbt = 4;   // bodies per tile (8: same time, more VGPRs)
    const int vt = (a.V + 255) / 256, nbt = (a.B + sbt - 1) / sbt;
    // about 4 workgroups per CU, each walking a run of body tiles
    int runs = (4 * (a.ncu > 0 ? a.ncu : 256) + vt - 1) / vt;
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
