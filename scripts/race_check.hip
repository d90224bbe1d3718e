// race_check.hip — determinism check of ONE DMA-path launch under load:
// runs the launch once for a reference output, then REPS more times and
// counts output halves that differ bitwise from the reference. Meant to be
// run while other processes load the GPU (scripts/gpu_race.sh).
//
//   race_check KIND LAYER REPS     KIND: G (cgemm3 graph), T (tgemm), S (stblock, layer 1)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "cgemm3.h"

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef unsigned short half_t;

static half_t* dev_halves(size_t n, unsigned seed) {
    std::vector<half_t> h(n);
    for (size_t i = 0; i < n; ++i) {
        seed = seed * 1664525u + 1013904223u;
        const float v = ((seed >> 9) & 0x3FFF) / 16384.0f - 0.5f;
        h[i] = __builtin_bit_cast(half_t, (_Float16)(v * 0.1f));
    }
    half_t* d;
    CK(hipMalloc(&d, n * 2));
    CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
    return d;
}

static float* dev_floats(size_t n, float v) {
    std::vector<float> h(n, v);
    float* d;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}

__global__ void diff_kernel(const unsigned* a, const unsigned* b, size_t n, unsigned long long* cnt) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long c = 0;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) c += a[i] != b[i];
    if (c) atomicAdd(cnt, c);
}

int main(int argc, char** argv) {
    const char kind = argc > 1 ? argv[1][0] : 'T';
    const int l = argc > 2 ? atoi(argv[2]) : 3;
    const int reps = argc > 3 ? atoi(argv[3]) : 200;
    const int N = 1024, T0 = 64, V = 17;
    struct L { int cin, cout, stride; };
    const L layers[8] = {{4, 64, 1}, {64, 64, 1}, {64, 128, 2}, {128, 128, 1},
                         {128, 128, 1}, {128, 128, 2}, {128, 256, 2}, {256, 256, 2}};
    int tin = T0;
    for (int i = 0; i < l; ++i) tin = (tin - 1) / layers[i].stride + 1;
    const L& Ly = layers[l];
    const int to = (tin - 1) / Ly.stride + 1;
    const long long rin = (long long)N * tin * V, rout = (long long)N * to * V;
    const int nbi = tik::sb_blocks(Ly.cin), nbo = tik::sb_blocks(Ly.cout);
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    half_t* x = dev_halves(rin * 64 * nbi, 1);
    half_t* z = dev_halves(rin * 64 * nbo, 2);
    half_t* o = dev_halves(rin * 64 * nbo, 3);
    half_t* ref = dev_halves(rin * 64 * nbo, 5);
    half_t* wsb = dev_halves(256 * 3 * 8 * 64, 4);
    half_t* zeros;
    CK(hipMalloc(&zeros, 256));
    CK(hipMemset(zeros, 0, 256));
    float* bias = dev_floats(V * 256, 0.01f);
    float* amix = dev_floats(V * V, 0.05f);
    unsigned long long* cnt;
    CK(hipMalloc(&cnt, 8));

    tik::Cgemm3Args g{};
    g.M = (int)rin; g.Nc = Ly.cout; g.V = V; g.tout = tin;
    g.seg[0] = tik::Seg3{x, nbi, 64 * nbi, 1, 1, 0, tin, wsb, 64 * nbi};
    g.nseg = 1; g.bias = bias; g.out_h = o; g.ldo = 64 * nbo; g.amix = amix;
    g.act = 1; g.mix_sparse = 1; g.zeros = zeros;
    tik::Cgemm3Args t{};
    t.M = (int)rout; t.Nc = Ly.cout; t.V = V; t.tout = to;
    t.seg[0] = tik::Seg3{z, nbo, 64 * nbo, 3, Ly.stride, 1, tin, wsb, 3 * 64 * nbo};
    t.nseg = 1;
    if (Ly.cin != Ly.cout || Ly.stride != 1) {
        t.seg[1] = tik::Seg3{x, nbi, 64 * nbi, 1, Ly.stride, 0, tin, wsb, 64 * nbi};
        t.nseg = 2;
    } else {
        t.resid = x; t.ldr = 64 * nbi;
    }
    t.bias = bias; t.out_h = o; t.ldo = 64 * nbo; t.act = 1; t.zeros = zeros;
    tik::StbArgs s{};
    s.x = x; s.ldx = 64 * nbi; s.nwin = N; s.T = tin; s.wg = wsb; s.ldwg = 64 * nbi; s.bias2 = bias; s.amix = amix;
    s.mix_sparse = 1; s.wt = wsb; s.ldwt = 3 * 64 * nbo; s.bias = bias; s.resid = 1; s.out = o; s.ldo = 64 * nbo;

    // head Linear 4352 -> 512 (H) and layer-0 temporal conv with the raw residual conv (R)
    tik::Cgemm3Args h{};
    const int hrows = N * 4;
    half_t* feat = kind == 'H' ? dev_halves((size_t)hrows * 64 * 136, 6) : nullptr;
    half_t* w0 = kind == 'H' ? dev_halves((size_t)512 * 64 * 136, 7) : nullptr;
    h.M = hrows; h.Nc = 512; h.V = 1; h.tout = hrows;
    h.seg[0] = tik::Seg3{feat, 136, 64 * 136, 1, 1, 0, hrows, w0, 64 * 136};
    h.nseg = 1; h.bias = bias; h.out_h = o; h.ldo = 64 * 16; h.act = 2; h.zeros = zeros;
    float* rx = kind == 'R' ? dev_floats((size_t)rin * 4, 0.3f) : nullptr;
    float* rw = kind == 'R' ? dev_floats(64 * 3, 0.2f) : nullptr;
    if (kind == 'R') {
        t.seg[1] = tik::Seg3{}; t.nseg = 1; t.resid = nullptr; t.rx = rx; t.rxc = 3; t.rw = rw;
    }
    // layer-0 spatial half from raw keypoints (Z): gcn0
    float* xr = kind == 'Z' ? dev_floats((size_t)rin * 3, 0.f) : nullptr;
    float* xb4 = kind == 'Z' ? dev_floats((size_t)rin * 4, 0.f) : nullptr;
    float* wg0 = kind == 'Z' ? dev_floats(64 * 4, 0.f) : nullptr;
    float* bnsc = kind == 'Z' ? dev_floats(17 * 3, 1.1f) : nullptr;
    float* bnsh = kind == 'Z' ? dev_floats(17 * 3, 0.05f) : nullptr;
    if (kind == 'Z') {
        std::vector<float> h((size_t)rin * 3);
        unsigned sd = 9;
        for (auto& v : h) { sd = sd * 1664525u + 1013904223u; v = ((sd >> 9) & 0x3FFF) / 16384.0f - 0.5f; }
        CK(hipMemcpy(xr, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> w(64 * 4);
        for (auto& v : w) { sd = sd * 1664525u + 1013904223u; v = ((sd >> 9) & 0x3FFF) / 16384.0f - 0.5f; }
        CK(hipMemcpy(wg0, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    }
    auto launch = [&]() {
        if (kind == 'Z') CK(tik::launch_gcn0(xr, (int)rin, V, 3, bnsc, bnsh, wg0, 4, bias, amix, 1, 64, o, 128, xb4, st));
        else if (kind == 'H') CK(tik::launch_cgemm3(h, tik::C3_H64x64, st));
        else if (kind == 'G') CK(tik::launch_cgemm3(g, Ly.cout % 128 ? tik::C3_G272x64 : tik::C3_G272x128_W8, st));
        else if (kind == 'S') CK(tik::launch_stblock(s, 64, 64, st));
        else CK(tik::launch_tgemm(t, Ly.cout >= 128 ? tik::TG_128x128 : tik::TG_128x64, st));
    };
    const size_t nout = kind == 'H' ? (size_t)hrows * 64 * 16 / 2 : (size_t)(kind == 'G' ? rin : rout) * 64 * nbo / 2;   // 32-bit words
    launch();
    CK(hipMemcpyAsync(ref, o, nout * 4, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
    if (argc > 4) {   // reference computed alone; wait for the load to start
        const double d = atof(argv[4]);
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < d) {}
    }
    unsigned long long total = 0, bad_reps = 0;
    for (int r = 0; r < reps; ++r) {
        CK(hipMemsetAsync(o, 0xFF, nout * 4, st));
        launch();
        CK(hipMemsetAsync(cnt, 0, 8, st));
        hipLaunchKernelGGL(diff_kernel, dim3(1024), dim3(256), 0, st, (const unsigned*)o, (const unsigned*)ref, nout, cnt);
        unsigned long long h = 0;
        CK(hipMemcpyAsync(&h, cnt, 8, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
        total += h;
        bad_reps += h != 0;
        if (h && bad_reps <= 3) {   // where: rows / halves that differ
            std::vector<unsigned> a(nout), b(nout);
            CK(hipMemcpy(a.data(), o, nout * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), ref, nout * 4, hipMemcpyDeviceToHost));
            const size_t wpr = (size_t)64 * nbo / 2;   // words per row
            long long r0 = -1, r1 = -1, nrow = 0, prev = -1;
            for (size_t i = 0; i < nout; ++i)
                if (a[i] != b[i]) {
                    const long long r = (long long)(i / wpr);
                    if (r0 < 0) r0 = r;
                    r1 = r;
                    if (r != prev) { ++nrow; prev = r; }
                }
            if (bad_reps == 1) {   // every differing word of the first bad rep: row, word, got, want
                int shown = 0;
                for (size_t i = 0; i < nout && shown < 400; ++i)
                    if (a[i] != b[i]) {
                        ++shown;
                        const half_t* ga = reinterpret_cast<const half_t*>(&a[i]);
                        const half_t* gb = reinterpret_cast<const half_t*>(&b[i]);
                        printf("    D %zu %zu %.6g %.6g %.6g %.6g\n", i / wpr, i % wpr,
                               (float)__builtin_bit_cast(_Float16, ga[0]), (float)__builtin_bit_cast(_Float16, gb[0]),
                               (float)__builtin_bit_cast(_Float16, ga[1]), (float)__builtin_bit_cast(_Float16, gb[1]));
                    }
            }
            size_t i0 = 0;
            while (a[i0] == b[i0]) ++i0;
            printf("  rep %d: %llu words in %lld rows, rows %lld..%lld; first word %zu (row %zu col-word %zu): got %08x want %08x\n", r, h,
                   nrow, r0, r1, i0, i0 / wpr, i0 % wpr, a[i0], b[i0]);
        }
    }
    printf("{\"kind\": \"%c\", \"layer\": %d, \"reps\": %d, \"bad_reps\": %llu, \"bad_words\": %llu, \"words\": %zu}\n", kind, l,
           reps, bad_reps, total, nout);
    return 0;
}
