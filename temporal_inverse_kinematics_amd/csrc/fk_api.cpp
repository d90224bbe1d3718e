// fk_api.cpp — C ABI of the SMPL-X FK check (include/tik.h, tik_fk_*).
// Replaces common/smpl_util.py:8-82 (load_smplx_models / run_smpl_inference)
// and the third-party smplx.SMPLX.forward it calls (lbs + landmarks).
//
// Per call (B bodies):
//   fk_chain            R_j, J, A_j, pose feature (B,512), first 55 joints (wave per body)
//   fk_blend            v_posed(B,3V) = [vec(R-I) | beta | expr | 1] . [posedirs; shapedirs; exprdirs; v_template]
//   fk_skin             T_v(b) = sum_j W[v][j] A_j(b); verts = T_v[:3,:3] v_posed + T_v[:,3] (+ transl)
//   fk_landmarks        21 vertex joints + 51 face landmarks + 17 dynamic contour landmarks
// bf16x3 (default): the blend shapes on xgemm.hip, the skinning on the sparse
// weights (fk.hip, at most 16 live joints per vertex, fp32 FMAs). Batches of
// more than one chunk (2048 bodies) run blend + skin per chunk, the chunks
// alternating between the caller's stream and a handle-owned one, so one
// chunk's HBM-bound skinning runs beside the next chunk's MFMA-bound blend
// shapes (a 2048-body v_posed is 257 MB, about the Infinity Cache); each
// chunk's landmarks follow its skinning in its stream.
// TIK_FK_SKIN=dense: the skinning as a GEMM on the persistent xgemm kernel
// (EPI_SKIN; also the path for weights with more than 16 live joints per
// vertex). fp32: both GEMMs on cgemm.hip.
// (Tried and not kept: the sparse skinning fused into the blend GEMM's
// epilogue, v_posed never in HBM: bitwise equal but 1.31 vs 0.91 ms, the
// per-tile A_j gather is latency-bound; profiles/r05_fk1_*. Also the blends in
// order on one stream with each chunk's skinning on the other: 1.01 vs 0.97 ms
// per 4096 bodies, a lone 2048-body blend takes 0.37 ms and two concurrent
// ones 0.56; profiles/r06_ab_fk_pipe.txt.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cgemm.h"
#include "common.h"
#include "fk.h"
#include "xgemm.h"

using namespace tik_host;

namespace {
constexpr int NJ = 55;
constexpr int KP = 512;   // padded blend-shape K (486 pose + 20 shape + 1 template)
constexpr int KJ = 64;    // padded skinning K (55 joints)
}  // namespace

struct tik_fk {
    int V = 0, F = 0, nb = 0, ne = 0, nlmk = 0, ndyn = 0, nextra = 0, njoints = 0;
    bool contour = false;
    DevBuf PT;         // [3V][KP]    (fp32 path)
    DevBuf WT;         // [V][KJ]     (fp32 path)
    DevHBuf xPT;       // bf16x3 tiles of P^T for xgemm.hip (the blend-shape GEMM, unfused paths)
    bool dense = false;   // TIK_FK_SKIN=dense: the skinning GEMM even when the weights are sparse
    // bodies per blend + skin chunk (TIK_FK_CHUNK at creation; >= B: one blend + one skin, the
    // round-4 arrangement). Same box, alternating (profiles/r06_fk_ab_chunk.txt): 2048 4.02-4.04M
    // bodies/s, 1024 3.93-3.95M, one chunk (4096) 3.91-3.95M
    int chunk = 2048;
    hipStream_t aux = nullptr;           // the second stream of the chunk pipeline
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    ~tik_fk() {
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        if (ev_join) (void)hipEventDestroy(ev_join);
        if (aux) (void)hipStreamDestroy(aux);
    }
    DevHBuf xWT;       // bf16x3 tiles of W^T for xgemm.hip (the dense skinning GEMM, EPI_SKIN)
    int ncu = 256;
    int prec = 2;
    // sparse skinning (fused, or fk.hip fk_skin_sparse_kernel): per vertex the joints with
    // W > 2^-30 as {joint, weight} pairs, sp_nz per vertex (0: more than 16, the dense GEMM)
    DevIBuf nzw;
    int sp_nz = 0;
    DevBuf jt, jd, pose_mean, lmk_bary, dyn_bary;
    DevIBuf parents, chain, faces, lmk_faces, dyn_faces, extra, depth;
    int nchain = 0, maxdepth = 0;
    int ldv = 0;       // v_posed row stride (3V rounded up to 4 floats: vector stores)
    // workspace
    DevBuf feat, ablk, vposed, verts_ws, ajt;
    DevHBuf trash;
    DevBuf zero_transl;   // (B,3) zeros: the skinning kernel always reads a translation
    DevIBuf dyn_bin;
    int cap = 0;
    Profiler prof;     // per-launch HIP events (tik_fk_profile; bench.py's FK roofline)
    bool profiling = false;
};

static const HostTensor* need(const TensorMap& m, const char* k, int& rc) {
    const HostTensor* t = find(m, k);
    if (!t) rc = fail(TIK_E_MISSING, "missing SMPL-X tensor '%s'", k);
    return t;
}

static std::vector<int> to_int(const HostTensor* t) {
    std::vector<int> o(t->v.size());
    for (size_t i = 0; i < o.size(); ++i) o[i] = (int)std::lround(t->v[i]);
    return o;
}

extern "C" {

int tik_fk_create(const tik_tensor* tensors, int n_tensors, int flags, tik_fk_t* out) {
    if (!tensors || n_tensors <= 0 || !out) return fail(TIK_E_INVALID, "tik_fk_create: null argument");
    *out = nullptr;
    TensorMap m = to_map(tensors, n_tensors);
    int rc = TIK_OK;
    const HostTensor* vt = need(m, "v_template", rc);
    const HostTensor* sd = need(m, "shapedirs", rc);
    const HostTensor* pd = need(m, "posedirs", rc);
    const HostTensor* jr = need(m, "J_regressor", rc);
    const HostTensor* lw = need(m, "lbs_weights", rc);
    const HostTensor* par = need(m, "parents", rc);
    const HostTensor* fc = need(m, "faces", rc);
    const HostTensor* lf = need(m, "lmk_faces_idx", rc);
    const HostTensor* lb = need(m, "lmk_bary_coords", rc);
    const HostTensor* ex = need(m, "extra_verts", rc);
    if (rc) return rc;
    const HostTensor* ed = find(m, "exprdirs");
    const HostTensor* pm = find(m, "pose_mean");
    const HostTensor* df = find(m, "dynamic_lmk_faces_idx");
    const HostTensor* db = find(m, "dynamic_lmk_bary_coords");
    auto* fk = new tik_fk();
    auto bad = [&](const char* msg) { delete fk; return fail(TIK_E_INVALID, "tik_fk_create: %s", msg); };
    if (vt->shape.size() != 2 || vt->shape[1] != 3) return bad("v_template must be (V,3)");
    const int V = fk->V = (int)vt->shape[0];
    if (sd->shape.size() != 3 || sd->shape[0] != V || sd->shape[1] != 3) return bad("shapedirs must be (V,3,nb)");
    fk->nb = (int)sd->shape[2];
    fk->ne = ed ? (int)ed->shape[2] : 0;
    if (ed && (ed->shape.size() != 3 || ed->shape[0] != V || ed->shape[1] != 3)) return bad("exprdirs must be (V,3,ne)");
    const int NS = fk->nb + fk->ne;
    if (54 * 9 + NS + 1 > KP || NS > 32) return bad("too many shape components");
    if (pd->shape.size() != 2 || pd->shape[0] != 54 * 9 || pd->shape[1] != 3 * V) return bad("posedirs must be (486, 3V)");
    if (jr->shape.size() != 2 || jr->shape[0] != NJ || jr->shape[1] != V) return bad("J_regressor must be (55,V)");
    if (lw->shape.size() != 2 || lw->shape[0] != V || lw->shape[1] != NJ) return bad("lbs_weights must be (V,55)");
    if ((int)par->v.size() != NJ) return bad("parents must have 55 entries");
    if (fc->shape.size() != 2 || fc->shape[1] != 3) return bad("faces must be (F,3)");
    fk->F = (int)fc->shape[0];
    fk->nlmk = (int)lf->v.size();
    fk->nextra = (int)ex->v.size();
    if ((int)lb->v.size() != 3 * fk->nlmk) return bad("lmk_bary_coords must be (L,3)");
    fk->contour = (flags & 1) && df && db;
    fk->ndyn = fk->contour ? (int)df->shape[1] : 0;
    if (fk->contour && (df->shape.size() != 2 || df->shape[0] != 79 || (int)db->v.size() != 79 * fk->ndyn * 3))
        return bad("dynamic_lmk_faces_idx must be (79,D), dynamic_lmk_bary_coords (79,D,3)");
    fk->njoints = NJ + fk->nextra + fk->nlmk + fk->ndyn;

    // index validation (host side, once)
    std::vector<int> hpar = to_int(par), hfaces = to_int(fc), hlf = to_int(lf), hex = to_int(ex);
    for (int j = 0; j < NJ; ++j)
        if (hpar[j] >= j || (j > 0 && hpar[j] < 0) || (j == 0 && hpar[j] != -1)) return bad("parents must be a topologically ordered tree rooted at 0");
    for (int f : hfaces) if (f < 0 || f >= V) return bad("face vertex index out of range");
    for (int f : hlf) if (f < 0 || f >= fk->F) return bad("landmark face index out of range");
    for (int v : hex) if (v < 0 || v >= V) return bad("extra vertex index out of range");
    std::vector<int> hdf;
    if (fk->contour) {
        hdf = to_int(df);
        for (int f : hdf) if (f < 0 || f >= fk->F) return bad("dynamic landmark face index out of range");
    }
    // depth of each joint in the tree: the chain kernel composes one level at a time
    std::vector<int> hdepth(NJ, 0);
    for (int j = 1; j < NJ; ++j) hdepth[j] = hdepth[hpar[j]] + 1;
    fk->maxdepth = *std::max_element(hdepth.begin(), hdepth.end());
    fk->ldv = (3 * V + 3) & ~3;
    // neck kinematic chain (smplx: from NECK_IDX=12 up to the root)
    std::vector<int> chain;
    for (int i = 12; i != -1; i = hpar[i]) chain.push_back(i);
    fk->nchain = (int)chain.size();

    // blend-shape matrix P^T (3V, KP): row 3v+c = [posedirs[:,3v+c] | shapedirs[v,c,:] | exprdirs[v,c,:] | v_template[v,c] | 0]
    std::vector<float> PT((size_t)3 * V * KP, 0.f);
    for (int v = 0; v < V; ++v)
        for (int c = 0; c < 3; ++c) {
            float* row = &PT[(size_t)(3 * v + c) * KP];
            for (int p = 0; p < 486; ++p) row[p] = pd->v[(size_t)p * 3 * V + 3 * v + c];
            for (int l = 0; l < fk->nb; ++l) row[486 + l] = sd->v[((size_t)v * 3 + c) * fk->nb + l];
            for (int l = 0; l < fk->ne; ++l) row[486 + fk->nb + l] = ed->v[((size_t)v * 3 + c) * fk->ne + l];
            row[486 + NS] = vt->v[(size_t)v * 3 + c];
        }
    std::vector<float> WT((size_t)V * KJ, 0.f);
    for (int v = 0; v < V; ++v)
        for (int j = 0; j < NJ; ++j) WT[(size_t)v * KJ + j] = lw->v[(size_t)v * NJ + j];
    // J_regressor folded into the template and blend shapes (float64 on the host)
    std::vector<float> jt(NJ * 3), jd((size_t)NJ * 3 * NS);
    for (int j = 0; j < NJ; ++j)
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            std::vector<double> d(NS, 0.0);
            for (int v = 0; v < V; ++v) {
                const double w = jr->v[(size_t)j * V + v];
                if (w == 0.0) continue;
                s += w * vt->v[(size_t)v * 3 + c];
                for (int l = 0; l < fk->nb; ++l) d[l] += w * sd->v[((size_t)v * 3 + c) * fk->nb + l];
                for (int l = 0; l < fk->ne; ++l) d[fk->nb + l] += w * ed->v[((size_t)v * 3 + c) * fk->ne + l];
            }
            jt[j * 3 + c] = (float)s;
            for (int l = 0; l < NS; ++l) jd[((size_t)j * 3 + c) * NS + l] = (float)d[l];
        }
    std::vector<float> hpm(NJ * 3, 0.f);
    if (pm) {
        if ((int)pm->v.size() != NJ * 3) return bad("pose_mean must be (55,3)");
        hpm = pm->v;
    }
    if ((rc = precision_from_env(fk->prec))) { delete fk; return rc; }
    if ((rc = fk->PT.upload(PT)) || (rc = fk->WT.upload(WT)) || (rc = fk->jt.upload(jt)) || (rc = fk->jd.upload(jd)) ||
        (rc = fk->pose_mean.upload(hpm)) || (rc = fk->lmk_bary.upload(lb->v)) || (rc = fk->parents.upload(hpar)) ||
        (rc = fk->chain.upload(chain)) || (rc = fk->faces.upload(hfaces)) || (rc = fk->lmk_faces.upload(hlf)) ||
        (rc = fk->extra.upload(hex)) || (rc = fk->depth.upload(hdepth))) {
        delete fk;
        return rc;
    }
    {   // sparse skinning weights
        const float tau = std::ldexp(1.0f, -30);
        int nzmax = 0;
        for (int v = 0; v < V; ++v) {
            int n = 0;
            for (int j = 0; j < NJ; ++j) n += lw->v[(size_t)v * NJ + j] > tau ? 1 : 0;
            nzmax = std::max(nzmax, n);
        }
        const int nz = nzmax <= 4 ? 4 : nzmax <= 8 ? 8 : nzmax <= 16 ? 16 : 0;
        const char* e = getenv("TIK_FK_SKIN");   // sparse (default) | dense
        fk->dense = e && !strcmp(e, "dense");
        if (const char* c = getenv("TIK_FK_CHUNK")) fk->chunk = std::max(1, atoi(c));
        if (nz && !fk->dense) {
            std::vector<int> h((size_t)V * nz * 2, 0);
            for (int v = 0; v < V; ++v) {
                int n = 0;
                for (int j = 0; j < NJ; ++j) {
                    const float w = lw->v[(size_t)v * NJ + j];
                    if (w > tau) {
                        h[((size_t)v * nz + n) * 2] = j;
                        std::memcpy(&h[((size_t)v * nz + n) * 2 + 1], &w, 4);
                        ++n;
                    }
                }
            }
            if ((rc = fk->nzw.upload(h))) {
                delete fk;
                return rc;
            }
            fk->sp_nz = nz;
        }
    }
    {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
            fk->ncu = n;
    }
    {
        const tik::XPackSeg ps{PT.data(), KP, 1, KP}, ws{WT.data(), KJ, 1, KJ};
        if ((rc = fk->xPT.upload(tik::xgemm_pack(&ps, 1, 3 * V, 128))) || (rc = fk->xWT.upload(tik::xgemm_pack(&ws, 1, V, 128)))) {
            delete fk;
            return rc;
        }
    }
    if (fk->contour && ((rc = fk->dyn_faces.upload(hdf)) || (rc = fk->dyn_bary.upload(db->v)))) {
        delete fk;
        return rc;
    }
    *out = fk;
    return TIK_OK;
}

int tik_fk_destroy(tik_fk_t fk) {
    delete fk;
    return TIK_OK;
}

int tik_fk_set_precision(tik_fk_t fk, int prec) {
    if (!fk || (prec != tik::PREC_F32 && prec != tik::PREC_BF16X3))
        return fail(TIK_E_INVALID, "tik_fk_set_precision: precision must be 0 (fp32) or 2 (bf16x3), got %d", prec);
    fk->prec = prec;
    return TIK_OK;
}

int tik_fk_num_joints(tik_fk_t fk) {
    if (!fk) return fail(TIK_E_INVALID, "null fk handle");
    return fk->njoints;
}

int tik_fk_num_verts(tik_fk_t fk) {
    if (!fk) return fail(TIK_E_INVALID, "null fk handle");
    return fk->V;
}

int tik_fk_reserve(tik_fk_t fk, int B) {
    if (!fk || B <= 0) return fail(TIK_E_INVALID, "tik_fk_reserve: bad arguments");
    if (B <= fk->cap) return TIK_OK;
    int rc;
    if ((rc = fk->feat.reserve((size_t)B * KP)) || (rc = fk->ablk.reserve((size_t)B * 16 * KJ)) ||
        (rc = fk->vposed.reserve((size_t)std::max(B, 2 * std::min(fk->chunk, B)) * fk->ldv)) || (rc = fk->dyn_bin.reserve((size_t)B)) ||
        (fk->sp_nz && (rc = fk->ajt.reserve((size_t)B * 55 * 12))) ||
        (rc = fk->zero_transl.upload(std::vector<float>((size_t)B * 3, 0.f))) ||
        (!fk->trash.p && (rc = fk->trash.upload(std::vector<unsigned short>(4096, 0)))))
        return rc;
    fk->cap = B;
    return TIK_OK;
}

int tik_fk_forward(tik_fk_t fk, const float* full_pose, const float* betas, const float* expression,
                   const float* transl, int B, float* joints, float* verts, void* stream) {
    if (!fk || !full_pose || !joints || B <= 0) return fail(TIK_E_INVALID, "tik_fk_forward: bad arguments");
    hipStream_t st = (hipStream_t)stream;
    int rc;
    if ((rc = tik_fk_reserve(fk, B))) return rc;
    float* vout = verts;
    if (!vout) {
        if ((rc = fk->verts_ws.reserve((size_t)B * 3 * fk->V))) return rc;
        vout = fk->verts_ws.p;
    }
    const bool bf = fk->prec == tik::PREC_BF16X3;
    tik::FkChainArgs c{};
    c.B = B; c.nb = fk->nb; c.ne = fk->ne; c.kp = KP; c.kj = KJ; c.njoints = fk->njoints; c.nchain = fk->nchain;
    c.pose = full_pose; c.betas = betas; c.expr = expression; c.transl = transl; c.pose_mean = fk->pose_mean.p;
    c.parents = fk->parents.p; c.chain = fk->chain.p; c.jt = fk->jt.p; c.jd = fk->jd.p;
    const bool sparse = bf && fk->sp_nz > 0;
    c.feat = fk->feat.p; c.ablk = sparse ? nullptr : fk->ablk.p;
    c.ajt = sparse ? fk->ajt.p : nullptr;
    // rows of A_j per body in ablk: the bf16x3 skinning GEMM skips the [0 0 0 1] row
    const int ar = bf ? 12 : 16;
    c.arows = ar;
    c.joints = joints; c.dyn_bin = fk->contour ? fk->dyn_bin.p : nullptr;
    c.depth = fk->depth.p; c.maxdepth = fk->maxdepth;
    Profiler* pf = fk->profiling ? &fk->prof : nullptr;
    const double Vd = fk->V;
    const int V3 = 3 * fk->V;
    const float* tr = transl ? transl : fk->zero_transl.p;
    {
        ProfRange pr(pf, "fk_chain", 0.0, 4.0 * (double)B * (NJ * 3 + 20 + KP + 16 * KJ), st);
        HIP_TRY(tik::launch_fk_chain(c, st));
    }

    // v_posed = feat . P on xgemm.hip (bf16x3, fp32 feat rows by LDS-DMA), bodies b0 .. b0 + n
    auto blend = [&](int b0, int n, float* vp, hipStream_t s) -> int {
        tik::XArgs g{};
        g.M = n; g.Nc = V3; g.V = 1; g.tout = n;
        g.seg[0] = tik::XSeg{fk->feat.p + (size_t)b0 * KP, KP, KP, 1, 1, 0, n, n};
        g.nseg = 1; g.wp = fk->xPT.p; g.ksteps = tik::xgemm_ksteps(g);
        g.out = vp; g.ldo = fk->ldv; g.act = tik::ACT_NONE; g.epi_lds = 1;
        // P^T (V3 x 512 bf16x3, ~97 MB) is the large operand: group the row tiles so each XCD
        // streams it about once (its contiguous run of workgroups covers gm row tiles x all columns)
        { const int gx = (n + 127) / 128; g.gm = (gx + 7) / 8; }
        // algorithmic: K = 507 live blend-shape columns (486 pose + 20 shape + template);
        // bytes: feat rows in, v_posed out, P^T once
        ProfRange pr(pf, "fk_blend", 2.0 * n * V3 * 507, 4.0 * ((double)n * KP + (double)n * V3 + (double)V3 * 507), s);
        HIP_TRY(tik::launch_xgemm(g, 128, tik::EPI_BIAS, s));
        return TIK_OK;
    };
    // skinning + vertex transform on the sparse weights (fk.hip): fp32 FMAs over each vertex's joints
    auto skin = [&](int b0, int n, const float* vp, hipStream_t s) -> int {
        tik::FkSkinSpArgs k{};
        k.B = n; k.V = fk->V; k.nz = fk->sp_nz; k.ajt = fk->ajt.p + (size_t)b0 * 12; k.ajt_ld = B;
        k.nzw = reinterpret_cast<const int2*>(fk->nzw.p);
        k.vposed = vp; k.ldv = fk->ldv; k.transl = tr + (size_t)b0 * 3; k.verts = vout + (size_t)b0 * V3;
        k.ncu = fk->ncu;
        // algorithmic: nz joints x 12 entries + the 3x4 vertex transform per (body, vertex);
        // bytes: A_j in, v_posed in, vertices out, the pairs once
        ProfRange pr(pf, "fk_skin", 2.0 * n * Vd * (12.0 * fk->sp_nz + 9.0),
                     4.0 * ((double)n * 12 * NJ + 2.0 * n * V3 + 2.0 * Vd * fk->sp_nz), s);
        HIP_TRY(tik::launch_fk_skin_sparse(k, s));
        return TIK_OK;
    };

    // the 21 vertex joints and 89 landmarks of bodies b0 .. b0 + n (after their vertices)
    auto lmk = [&](int b0, int n, hipStream_t s) -> int {
        tik::FkLmkArgs l{};
        l.B = n; l.V = fk->V; l.njoints = fk->njoints; l.nextra = fk->nextra; l.nlmk = fk->nlmk; l.ndyn = fk->ndyn;
        l.verts = vout + (size_t)b0 * V3; l.transl = transl ? transl + (size_t)b0 * 3 : nullptr;
        l.extra = fk->extra.p; l.faces = fk->faces.p; l.lmk_faces = fk->lmk_faces.p;
        l.lmk_bary = fk->lmk_bary.p; l.dyn_faces = fk->dyn_faces.p; l.dyn_bary = fk->dyn_bary.p;
        l.dyn_bin = fk->dyn_bin.p + b0; l.joints = joints + (size_t)b0 * fk->njoints * 3;
        ProfRange pr(pf, "fk_landmarks", 0.0, 4.0 * (double)n * (3.0 * 144 + 3.0 * 3 * 3 * 89), s);
        HIP_TRY(tik::launch_fk_landmarks(l, s));
        return TIK_OK;
    };

    if (sparse) {
        const int CH = fk->chunk, nch = (B + CH - 1) / CH;
        if (nch > 1 && !fk->aux) {
            HIP_TRY(hipStreamCreateWithFlags(&fk->aux, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&fk->ev_fork, hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&fk->ev_join, hipEventDisableTiming));
        }
        if (nch > 1) {
            HIP_TRY(hipEventRecord(fk->ev_fork, st));
            HIP_TRY(hipStreamWaitEvent(fk->aux, fk->ev_fork, 0));
        }
        for (int k = 0; k < nch; ++k) {
            const int b0 = k * CH, n = std::min(CH, B - b0);
            hipStream_t s = (k & 1) ? fk->aux : st;
            // two v_posed chunk buffers, one per stream (reused in stream order)
            float* vp = fk->vposed.p + (size_t)(nch > 1 ? (k & 1) * CH : 0) * fk->ldv;
            // each chunk's landmarks in its stream, beside the other stream's skinning
            if ((rc = blend(b0, n, vp, s)) || (rc = skin(b0, n, vp, s)) || (rc = lmk(b0, n, s))) return rc;
        }
        if (nch > 1) {
            HIP_TRY(hipEventRecord(fk->ev_join, fk->aux));
            HIP_TRY(hipStreamWaitEvent(st, fk->ev_join, 0));
        }
    } else if (bf) {
        if ((rc = blend(0, B, fk->vposed.p, st))) return rc;
        // skinning + vertex transform as a GEMM on the persistent xgemm kernel (EPI_SKIN): the DMA
        // pipeline runs across tiles (K = 64 is 2 steps per tile); rows = body * 12 + transform entry
        tik::XArgs s{};
        s.M = B * ar; s.Nc = fk->V; s.V = 1; s.tout = B * ar;
        s.seg[0] = tik::XSeg{fk->ablk.p, KJ, KJ, 1, 1, 0, B * ar, (long long)B * ar};
        s.nseg = 1; s.wp = fk->xWT.p; s.ksteps = tik::xgemm_ksteps(s); s.skin_rows = ar;
        s.resid = fk->vposed.p; s.ldr = fk->ldv; s.out = vout; s.ldo = V3; s.act = tik::ACT_NONE;
        s.bias = tr;
        s.trash = reinterpret_cast<float*>(fk->trash.p);
        // algorithmic: 12 transform entries x 55 joints per (body, vertex) + the
        // 3x4 vertex transform; bytes: A_j rows and v_posed in, vertices out, W once
        ProfRange pr(pf, "fk_skin", 2.0 * B * Vd * 12 * NJ + 18.0 * B * Vd,
                     4.0 * ((double)B * 12 * NJ + 2.0 * B * V3 + Vd * NJ), st);
        HIP_TRY(tik::launch_xgemm_pt(s, 128, fk->ncu, st, tik::EPI_SKIN));
    } else {
        {
            tik::CgemmArgs g{};   // v_posed = feat . P (exact fp32 MFMA)
            g.M = B; g.Nc = V3; g.V = 1; g.tout = B;
            g.seg[0] = tik::Seg{fk->feat.p, fk->PT.p, KP, KP, 1, 1, 0, B, KP};
            g.nseg = 1; g.out = fk->vposed.p; g.ldo = fk->ldv; g.act = tik::ACT_NONE;
            ProfRange pr(pf, "fk_blend", 2.0 * B * V3 * 507, 4.0 * ((double)B * KP + (double)B * V3 + (double)V3 * 507), st);
            HIP_TRY(tik::launch_cgemm(g, tik::CFG_T128x128, st, tik::PREC_F32));
        }
        tik::CgemmArgs s{};   // skinning + vertex transform (exact fp32 MFMA)
        s.M = B * 16; s.Nc = fk->V; s.V = 1; s.tout = B * 16;
        s.seg[0] = tik::Seg{fk->ablk.p, fk->WT.p, KJ, KJ, 1, 1, 0, B * 16, KJ};
        s.nseg = 1; s.resid = fk->vposed.p; s.ldr = fk->ldv; s.out = vout; s.ldo = V3; s.bias = transl;
        ProfRange pr(pf, "fk_skin", 2.0 * B * Vd * 16 * NJ + 18.0 * B * Vd,
                     4.0 * ((double)B * 16 * NJ + 2.0 * B * V3 + Vd * NJ), st);
        HIP_TRY(tik::launch_cgemm(s, tik::CFG_S128x128, st, tik::PREC_F32));
    }

    if (!sparse) return lmk(0, B, st);
    return TIK_OK;
}

int tik_fk_profile(tik_fk_t fk, int max_launches) {
    if (!fk || max_launches < 0) return fail(TIK_E_INVALID, "tik_fk_profile: bad arguments");
    fk->profiling = max_launches > 0;
    return max_launches > 0 ? fk->prof.enable(max_launches) : (fk->prof.clear(), TIK_OK);
}

int tik_fk_profile_count(tik_fk_t fk) {
    if (!fk) return fail(TIK_E_INVALID, "null FK handle");
    return (int)fk->prof.recs.size();
}

int tik_fk_profile_read(tik_fk_t fk, int i, char* label, int label_len, float* ms, double* flops, double* bytes) {
    if (!fk) return fail(TIK_E_INVALID, "tik_fk_profile_read: null FK handle");
    return fk->prof.read(i, label, label_len, ms, flops, bytes);
}

}  // extern "C"
