// kbench.hip — tile/pipeline tuning harness for the cgemm3 (f16x3, LDS-DMA)
// launches of the IK backbone at bench.py's size (1024 windows x 64 frames).
// Times every candidate config of every layer's G (gcn + graph mix) and T
// (tcn + residual) launch with HIP events; numbers only (parity lives in tests/).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/kbench.hip -Itemporal_inverse_kinematics_amd/csrc \
//       -Ltemporal_inverse_kinematics_amd -ltik -Wl,-rpath,$PWD/temporal_inverse_kinematics_amd -o build/kbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cgemm3.h"

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
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

static const char* cfg_name(int c) {
    static const char* n[] = {"T128x128", "T128x64",     "G272x64",     "H64x64",      "T128x128_S3", "T128x128_S4",
                              "T256x128_W8", "T256x64_W8", "T128x64_S4", "G272x128_W8", "G272x64_S2",
                              "dbg128x128_DMA", "dbg128x128_MFMA", "dbg128x64_DMA", "dbg128x64_MFMA"};
    return c < tik::C3_NCFG ? n[c] : "?";
}

static float time_launch(const tik::Cgemm3Args& a, int cfg, hipStream_t st, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) CK(tik::launch_cgemm3(a, cfg, st));
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) CK(tik::launch_cgemm3(a, cfg, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 1024, T0 = argc > 2 ? atoi(argv[2]) : 64;
    const int reps = argc > 3 ? atoi(argv[3]) : 20, V = 17;
    struct L { int cin, cout, stride; };
    const L layers[8] = {{8, 64, 1}, {64, 64, 1}, {64, 128, 2}, {128, 128, 1},
                         {128, 128, 1}, {128, 128, 2}, {128, 256, 2}, {256, 256, 2}};
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const size_t maxrows = (size_t)N * T0 * V;
    half_t* x = dev_halves(maxrows * 256 * 2, 1);
    half_t* z = dev_halves(maxrows * 256 * 2, 2);
    half_t* o = dev_halves(maxrows * 256 * 2, 3);
    half_t* wh = dev_halves(256 * 3 * 256, 4);
    half_t* wl = dev_halves(256 * 3 * 256, 5);
    half_t* zeros;
    CK(hipMalloc(&zeros, 256));
    CK(hipMemset(zeros, 0, 256));
    float* bias = dev_floats(V * 256, 0.01f);
    float* amix = dev_floats(V * V, 0.05f);
    int tin = T0;
    double tot_best = 0, tot_cur = 0;
    for (int l = 0; l < 8; ++l) {
        const L& Ly = layers[l];
        const int to = (tin - 1) / Ly.stride + 1;
        const long long rin = (long long)N * tin * V, rout = (long long)N * to * V;
        tik::Cgemm3Args g{};
        g.M = (int)rin; g.Nc = Ly.cout; g.V = V; g.tout = tin;
        g.seg[0] = tik::Seg3{x, rin * Ly.cin, Ly.cin, Ly.cin, 1, 1, 0, tin, wh, wl, Ly.cin};
        g.nseg = 1; g.bias = bias; g.out_h = z; g.out_plane = rin * Ly.cout; g.ldo = Ly.cout; g.amix = amix;
        g.act = 1; g.mix_sparse = 1; g.zeros = zeros;
        const int gc[] = {tik::C3_G272x64, tik::C3_G272x128_W8};
        const double gbytes = 4.0 * (rin * Ly.cin + rin * Ly.cout);
        float best = 1e9, cur = 0;
        for (int c : gc) {
            if (c == tik::C3_G272x128_W8 && Ly.cout % 128) continue;
            const float ms = time_launch(g, c, st, reps);
            if (c == tik::C3_G272x64) cur = ms;
            if (ms < best) best = ms;
            printf("L%d G %-12s %8.4f ms  %6.0f GB/s\n", l, cfg_name(c), ms, gbytes / ms / 1e6);
        }
        tot_best += best; tot_cur += cur;
        tik::Cgemm3Args t{};
        t.M = (int)rout; t.Nc = Ly.cout; t.V = V; t.tout = to;
        t.seg[0] = tik::Seg3{z, rin * Ly.cout, Ly.cout, Ly.cout, 3, Ly.stride, 1, tin, wh, wl, 3 * Ly.cout};
        t.nseg = 1;
        if (Ly.cin != Ly.cout || Ly.stride != 1) {
            t.seg[1] = tik::Seg3{x, rin * Ly.cin, Ly.cin, Ly.cin, 1, Ly.stride, 0, tin, wh, wl, Ly.cin};
            t.nseg = 2;
        } else {
            t.resid = x; t.resid_plane = rin * Ly.cin; t.ldr = Ly.cin;
        }
        t.bias = bias; t.out_h = o; t.out_plane = rout * Ly.cout; t.ldo = Ly.cout; t.act = 1; t.zeros = zeros;
        const double tfl = 2.0 * rout * Ly.cout * (3.0 * Ly.cout + (t.nseg > 1 ? Ly.cin : 0));
        std::vector<int> tc;
        if (Ly.cout >= 128) tc = {tik::C3_T128x128, tik::C3_T256x128_W8, tik::C3_DBG_T128x128_DMA, tik::C3_DBG_T128x128_MFMA};
        else tc = {tik::C3_T128x64, tik::C3_T256x64_W8, tik::C3_DBG_T128x64_DMA, tik::C3_DBG_T128x64_MFMA};
        best = 1e9; cur = 0;
        for (int c : tc) {
            const float ms = time_launch(t, c, st, reps);
            if (c == tc[0]) cur = ms;
            if (ms < best && c < tik::C3_DBG_T128x128_DMA) best = ms;
            printf("L%d T %-12s %8.4f ms  %6.1f TF(fp32-eq)\n", l, cfg_name(c), ms, tfl / ms / 1e9);
        }
        tot_best += best; tot_cur += cur;
        tin = to;
    }
    printf("backbone G+T: current configs %.4f ms, best-per-launch %.4f ms\n", tot_cur, tot_best);
    return 0;
}
