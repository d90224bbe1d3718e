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
    float* feat;             // (B,kp)  [vec(R_j - I), j=1..54 | betas | expr | 1 | 0..]
    float* ablk;             // (B,16,kj) rows e = 4r+c of A_j (3x4), cols j
    float* joints;           // (B,njoints,3): first 55 written here
    int* dyn_bin;            // (B) or null
};

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
