// common.h — host-side helpers shared by the C-ABI translation units:
// thread-local last error, HIP error mapping, owning device buffers and the
// state-dict view of a tik_tensor array.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/tik.h"

namespace tik_host {

extern thread_local std::string g_err;

inline int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}


#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(TIK_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

constexpr float BN_EPS = 1e-5f;
constexpr int TK = 3;   // temporal kernel (pose_trainer.py:85)

struct HostTensor {
    std::vector<float> v;
    std::vector<int64_t> shape;
};

using TensorMap = std::map<std::string, HostTensor>;

inline TensorMap to_map(const tik_tensor* t, int n) {
    TensorMap m;
    for (int i = 0; i < n; ++i) {
        if (!t[i].name) continue;
        HostTensor h;
        int64_t numel = 1;
        for (int d = 0; d < t[i].ndim; ++d) {
            h.shape.push_back(t[i].shape[d]);
            numel *= t[i].shape[d];
        }
        if (t[i].data) h.v.assign(t[i].data, t[i].data + numel);
        m[t[i].name] = std::move(h);
    }
    return m;
}

inline const HostTensor* find(const TensorMap& m, const std::string& k) {
    auto it = m.find(k);
    return it == m.end() ? nullptr : &it->second;
}

// Debug hook (TIK_GUARD=1): every device buffer gets 1 MiB guard zones on
// both sides filled with 0xA5; tik_debug_check_guards() reports the first
// buffer whose guards were written (an out-of-bounds store).
constexpr size_t GUARD_BYTES = 1 << 20;
bool guard_mode();
void guard_register(void* base, size_t bytes);
void guard_unregister(void* base);

inline hipError_t dev_alloc(void** p, size_t bytes) {
    if (!guard_mode()) return hipMalloc(p, bytes);
    char* base = nullptr;
    const size_t tot = bytes + 2 * GUARD_BYTES;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&base), tot);
    if (e != hipSuccess) return e;
    if ((e = hipMemset(base, 0xA5, tot)) != hipSuccess) return e;
    guard_register(base, bytes);
    *p = base + GUARD_BYTES;
    return hipSuccess;
}
inline void dev_free(void* p) {
    if (!p) return;
    if (!guard_mode()) { (void)hipFree(p); return; }
    char* base = static_cast<char*>(p) - GUARD_BYTES;
    guard_unregister(base);
    (void)hipFree(base);
}

template <class T>
struct DevArray {   // owning device buffer; move-only (a copy would double-free)
    T* p = nullptr;
    size_t n = 0;
    DevArray() = default;
    DevArray(const DevArray&) = delete;
    DevArray& operator=(const DevArray&) = delete;
    DevArray(DevArray&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevArray& operator=(DevArray&& o) noexcept {
        if (this != &o) {
            dev_free(p);
            p = o.p; n = o.n; o.p = nullptr; o.n = 0;
        }
        return *this;
    }
    ~DevArray() { dev_free(p); }
    int upload(const std::vector<T>& h) {
        dev_free(p); p = nullptr;
        n = h.size();
        if (n == 0) return TIK_OK;
        if (dev_alloc(reinterpret_cast<void**>(&p), n * sizeof(T)) != hipSuccess) { n = 0; return fail(TIK_E_NOMEM, "hipMalloc(%zu elements) failed", h.size()); }
        if (hipMemcpy(p, h.data(), n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
            return fail(TIK_E_HIP, "hipMemcpy H2D failed");
        return TIK_OK;
    }
    int reserve(size_t want) {
        if (want <= n) return TIK_OK;
        dev_free(p); p = nullptr;
        if (dev_alloc(reinterpret_cast<void**>(&p), want * sizeof(T)) != hipSuccess) { n = 0; return fail(TIK_E_NOMEM, "hipMalloc(%zu elements) failed", want); }
        n = want;
        return TIK_OK;
    }
};
using DevBuf = DevArray<float>;
using DevIBuf = DevArray<int>;
using DevHBuf = DevArray<unsigned short>;

// fp32 -> bf16 bits, round to nearest even (finite inputs; NaN stays NaN)
inline unsigned short bf16_rne(float x) {
    unsigned u;
    memcpy(&u, &x, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (unsigned short)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
    return (unsigned short)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
inline float bf16_to_f32(unsigned short b) {
    const unsigned u = (unsigned)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
// x = p0 + p1 + p2 with p_i = bf16_rne(x - p0 - ... - p_{i-1}): exact for
// normal fp32 x (each plane takes the next 8 significant bits, the
// residuals are exact in fp32), full fp32 exponent range
inline void split_bf16x3(float x, unsigned short& p0, unsigned short& p1, unsigned short& p2) {
    p0 = bf16_rne(x);
    const float r1 = x - bf16_to_f32(p0);
    p1 = bf16_rne(r1);
    const float r2 = r1 - bf16_to_f32(p1);
    p2 = bf16_rne(r2);
}

// fp32 weights [Nc][kt][cin] (row stride ldw floats) -> three bf16 planes
// [Nc][kt][cin8] (cin8 = cin rounded up to 8, zero-filled): w = p0 + p1 + p2
// (split_bf16x3). The PREC_BF16X3 arithmetic of cgemm.hip.
struct SplitW3 {
    DevHBuf p[3];
    int cin8 = 0, ldw8 = 0;
    int build(const std::vector<float>& w, int Nc, int kt, int cin, int ldw) {
        cin8 = (cin + 7) & ~7;
        ldw8 = kt * cin8;
        std::vector<unsigned short> h[3];
        for (auto& v : h) v.assign((size_t)Nc * ldw8, 0);
        for (int n = 0; n < Nc; ++n)
            for (int t = 0; t < kt; ++t)
                for (int c = 0; c < cin; ++c) {
                    const size_t o = (size_t)n * ldw8 + (size_t)t * cin8 + c;
                    split_bf16x3(w[(size_t)n * ldw + (size_t)t * cin + c], h[0][o], h[1][o], h[2][o]);
                }
        int rc;
        for (int i = 0; i < 3; ++i)
            if ((rc = p[i].upload(h[i]))) return rc;
        return TIK_OK;
    }
};

// default arithmetic of the GEMMs (cgemm.h PREC_*): TIK_PRECISION=fp32 the
// exact f32 MFMA path; unset or bf16x3, the 6-product bf16 split with fp32's
// exponent range. Any other value fails the handle's creation (f16x3 was
// retired in round 5: silently mapping it to bf16x3 would change the
// arithmetic without a word)
inline int precision_from_env(int& prec) {
    const char* e = getenv("TIK_PRECISION");
    const std::string s = e ? e : "";
    if (s.empty() || s == "bf16x3") prec = 2;
    else if (s == "fp32" || s == "f32") prec = 0;
    else if (s == "f16x3") return fail(TIK_E_INVALID, "TIK_PRECISION=f16x3 was retired (round 5); use bf16x3 or fp32");
    else return fail(TIK_E_INVALID, "TIK_PRECISION=%s: expected bf16x3 or fp32", s.c_str());
    return TIK_OK;
}

// One set of activation buffers for the IK forward. A model handle owns two
// (the caller-stream half and the aux-stream half of a split batch); every
// online-IK stream owns its own, so a batch call on the handle can never
// reallocate or overwrite memory a captured stream graph points at.
struct Workspace {
    DevBuf xb, z, a0, a1, hid;       // layer-0 residual input, z, activation ping-pong, head hidden
    DevBuf z2;                       // the second z of fused launches (xtws FG: block l+1's z beside block l's)
    DevBuf part;                     // split-K partial sums (small-batch launches)
};

// Optional per-launch HIP-event profiler (bench.py's roofline numbers): one
// event pair per kernel launch on the launch stream, algorithmic FLOPs and
// bytes computed from the shapes.
struct Profiler {
    struct Rec {
        std::string label;
        double flops, bytes;
    };
    std::vector<hipEvent_t> ev0, ev1;
    std::vector<Rec> recs;
    int cap = 0;
    ~Profiler() { clear(); }
    void clear() {
        for (auto e : ev0) (void)hipEventDestroy(e);
        for (auto e : ev1) (void)hipEventDestroy(e);
        ev0.clear(); ev1.clear(); recs.clear(); cap = 0;
    }
    int enable(int n) {
        clear();
        for (int i = 0; i < n; ++i) {
            hipEvent_t a, b;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)
                return fail(TIK_E_HIP, "hipEventCreate failed");
            ev0.push_back(a); ev1.push_back(b);
        }
        cap = n;
        return TIK_OK;
    }
    int begin(const char* label, double flops, double bytes, hipStream_t st) {
        if ((int)recs.size() >= cap) return -1;
        const int i = (int)recs.size();
        recs.push_back({label, flops, bytes});
        (void)hipEventRecord(ev0[i], st);
        return i;
    }
    void end(int i, hipStream_t st) {
        if (i >= 0) (void)hipEventRecord(ev1[i], st);
    }
    // record i's label, HIP-event time and algorithmic work (after the stream synchronised)
    int read(int i, char* label, int label_len, float* ms, double* flops, double* bytes) const {
        if (i < 0 || i >= (int)recs.size()) return fail(TIK_E_INVALID, "profile read: bad index %d", i);
        const auto& r = recs[i];
        if (label && label_len > 0) {
            strncpy(label, r.label.c_str(), label_len - 1);
            label[label_len - 1] = 0;
        }
        if (flops) *flops = r.flops;
        if (bytes) *bytes = r.bytes;
        if (ms) HIP_TRY(hipEventElapsedTime(ms, ev0[i], ev1[i]));
        return TIK_OK;
    }
};

// one profiled launch: the event pair around the scope (no-op when p is null)
struct ProfRange {
    Profiler* p;
    hipStream_t st;
    int i;
    ProfRange(Profiler* p_, const char* label, double flops, double bytes, hipStream_t s)
        : p(p_), st(s), i(p_ ? p_->begin(label, flops, bytes, s) : -1) {}
    ~ProfRange() { if (p) p->end(i, st); }
};

}  // namespace tik_host

struct tik_model;
namespace tik { struct OnlineArgs; }
namespace tik_host {
// internal entry points shared by api.cpp and stream.cpp
int model_reserve_ws(tik_model* m, Workspace& w, int N, int T);
// the IK forward on workspace w; split = may run as two halves on two streams
int model_forward_ws(tik_model* m, const float* x, int N, int T, float* poses, hipStream_t st, Workspace& w,
                     bool split);
void model_retain(tik_model* m);    // a stream keeps its model alive
void model_release(tik_model* m);   // deletes the model at the last reference
// the fp32 weights and shapes of the online-IK dataflow kernel (online.h);
// TIK_E_INVALID when the model is outside what that kernel supports
int model_online_fill(tik_model* m, tik::OnlineArgs& a);
int model_pose_dim(const tik_model* m);   // 0 for a backbone-only handle


}  // namespace tik_host
