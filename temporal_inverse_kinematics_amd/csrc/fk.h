#pragma once
#include <hip/hip_runtime.h>

namespace tik {

struct FkChainArgs {
    int B, nb, ne, kp, kj, njoints, nchain;
    const float* pose;       // (B,55,3)
    const float* betas;      // (B,nb) or null
    const float* expr;       // (B,ne) or null
    const float* transl;     // (B,3) or null
    const float* pose_mean;  // (55,3)
    const int* parents;      // (55)
    const int* chain;        // neck kinematic chain (nchain)
    const float* jt;         // (55,3)        J_regressor . v_template
    const float* jd;         // (55,3,nb+ne)  J_regressor . [shapedirs | exprdirs]
    float* feat;             // (B,kp)  [vec(R_j - I), j=1..54 | betas | expr | 1 | 0..]  (fp32 GEMM path; or null)
    float* ablk;             // (B,arows,kj) rows e = 4r+c of A_j (3x4), cols j                (fp32 GEMM path; or null)
    int arows;               // rows of ablk per body: 16 (rows 12..15 = [0 0 0 1]) or 12 (the 3x4 part only)
    float* ajt;              // (55,B,12) A_j joint-major for the sparse / fused skinning (or null)
    float* joints;           // (B,njoints,3): first 55 written here
    int* dyn_bin;            // (B) or null
    const int* depth;        // (55) depth of each joint in the kinematic tree (root 0)
    int maxdepth;
};

// LBS on the sparse skinning weights: T = sum over the (at most nz)
// joints of vertex v with W[v][j] > 2^-30, in ascending joint order, in fp32
// FMAs (the dense product's terms in its order, minus terms below 2^-30 of a
// transform); one thread per vertex, a run of bodies per workgroup.
struct FkSkinSpArgs {
    int B, V, nz;                    // nz: entries per vertex (4, 8 or 16)
    const float* ajt;                // A_j joint-major: body b, joint j at ajt[(j * ajt_ld + b) * 12]
    int ajt_ld;                      // bodies per joint row of ajt (>= B: a chunk of a larger batch)
    const int2* nzw;                 // (V,nz) {joint, float bits of W[v][joint]}, joints ascending; padding {0, 0}
    const float* vposed;             // (B, ldv) v_posed, 3V used
    int ldv;
    const float* transl;             // (B,3): a zero array when the caller has none
    float* verts;                    // (B, 3V)
    int ncu;
};
hipError_t launch_fk_skin_sparse(const FkSkinSpArgs& a, hipStream_t st);

struct FkLmkArgs {
    int B, V, njoints, nextra, nlmk, ndyn;
    const float* verts;      // (B,V,3) including transl
    const float* transl;     // (B,3) or null
    const int* extra;        // (nextra)
    const int* faces;        // (F,3)
    const int* lmk_faces;    // (nlmk)
    const float* lmk_bary;   // (nlmk,3)
    const int* dyn_faces;    // (79,ndyn)
    const float* dyn_bary;   // (79,ndyn,3)
    const int* dyn_bin;      // (B)
    float* joints;           // (B,njoints,3): rows 55.. written here
};

hipError_t launch_fk_chain(const FkChainArgs& a, hipStream_t st);
hipError_t launch_fk_landmarks(const FkLmkArgs& a, hipStream_t st);

}  // namespace tik
