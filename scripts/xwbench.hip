// xwbench.hip — timing harness for the 128-channel stride-1 temporal conv
// (xtws.hip) with and without the fused next-block gcn (FG), beside the
// standalone gcn (xgraph.hip), at bench.py's L3 size (1024 windows x 32
// frames). Diagnostic build: the kernels are compiled in with -DTIK_XTUNE
// (parts switched off by XTConvArgs::tune bits) and -DTIK_XTRACE (per-phase
// s_memtime sums of waves 0 and 4). Numbers only; parity lives in tests/.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DTIK_XTUNE -DTIK_XTRACE -Iinclude \
//       -Itemporal_inverse_kinematics_amd/csrc scripts/xwbench.hip \
//       temporal_inverse_kinematics_amd/csrc/xtws.hip temporal_inverse_kinematics_amd/csrc/xgraph.hip -o build/xwbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "xgraph.h"
#include "xtws.h"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

template <class T>
static T* dev_fill(size_t n, unsigned seed, float scale, bool bf16) {
    std::vector<T> h(n);
    for (size_t i = 0; i < n; ++i) {
        seed = seed * 1664525u + 1013904223u;
        const float v = (((seed >> 9) & 0x3FFF) / 16384.0f - 0.5f) * scale;
        if (bf16) {
            unsigned u;
            memcpy(&u, &v, 4);
            h[i] = (T)(u >> 16);
        } else {
            h[i] = (T)v;
        }
    }
    T* d;
    CK(hipMalloc(&d, n * sizeof(T)));
    CK(hipMemcpy(d, h.data(), n * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

template <class F>
static float time_ms(F&& launch, hipStream_t st, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) CK(launch());
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) CK(launch());
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 1024, T = argc > 2 ? atoi(argv[2]) : 32, reps = argc > 3 ? atoi(argv[3]) : 20;
    const int V = 17, C = 128, M = N * T * V;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    float* z = dev_fill<float>((size_t)M * C, 1, 2.f, false);
    float* x = dev_fill<float>((size_t)M * C, 2, 2.f, false);
    float* out = dev_fill<float>((size_t)M * C, 3, 0.f, false);
    float* z2 = dev_fill<float>((size_t)M * C, 4, 0.f, false);
    unsigned short* wt = dev_fill<unsigned short>((size_t)8 * 12 * 3 * 64 * 8, 5, 0.05f, true);
    unsigned short* wg = dev_fill<unsigned short>((size_t)8 * 4 * 3 * 64 * 8, 6, 0.05f, true);
    float* bias = dev_fill<float>(C, 7, 0.1f, false);
    float* bias2 = dev_fill<float>(V * C, 8, 0.1f, false);
    float* amix = dev_fill<float>(V * V, 9, 0.2f, false);
    float* trash = dev_fill<float>(4096, 10, 0.f, false);
    unsigned long long* trace;
    CK(hipMalloc(&trace, (size_t)ncu * 16 * 8));

    tik::XTConvArgs c{};
    c.M = M; c.T = T; c.z = z; c.ldz = C; c.x = x; c.ldx = C; c.wp = wt; c.bias = bias; c.out = out; c.ldo = C;
    c.nts = 1; c.trash = trash;
    tik::XGraphArgs g{};
    g.nframes = N * T; g.x = out; g.ldx = C; g.cin = C; g.cout = C; g.wp = wg; g.bias2 = bias2; g.amix = amix;
    g.mix_sparse = 1; g.out = z2; g.ldo = C; g.nts = 1; g.trash = trash;
    const float t_xtw = time_ms([&] { return tik::launch_xtws(c, ncu, st); }, st, reps);
    const float t_xgw = time_ms([&] { return tik::launch_xgraph(g, ncu, st); }, st, reps);
    printf("XTW %.4f ms  XGW %.4f ms  sum %.4f ms\n", t_xtw, t_xgw, t_xtw + t_xgw);
    tik::XTConvArgs f = c;
    f.wg = wg; f.bias2 = bias2; f.amix = amix; f.mix_sparse = 1; f.zout = z2; f.ldzo = C;
    const int masks[] = {0, 16, 32, 64, 16 | 32, 16 | 32 | 64, 4, 4 | 16, 1 | 2 | 4 | 8 | 16 | 32 | 64};
    for (int m : masks) {
        f.tune = m;
        printf("XTWG tune %3d %.4f ms\n", m, time_ms([&] { return tik::launch_xtws(f, ncu, st); }, st, reps));
    }
    // phase trace of the default fused launch
    f.tune = 0;
    f.trace = trace;
    CK(hipMemset(trace, 0, (size_t)ncu * 16 * 8));
    CK(tik::launch_xtws(f, ncu, st));
    CK(hipStreamSynchronize(st));
    std::vector<unsigned long long> h((size_t)ncu * 16);
    CK(hipMemcpy(h.data(), trace, h.size() * 8, hipMemcpyDeviceToHost));
    double s0[8] = {0}, s4[8] = {0}, tiles = 0;
    for (int w = 0; w < ncu; ++w) {
        const unsigned long long nt = h[16 * w + 7] >> 48;
        if (!nt) continue;
        tiles += (double)nt;
        for (int k = 0; k < 8; ++k) {
            s0[k] += (double)(k == 7 ? (h[16 * w + 7] & ((1ull << 48) - 1)) : h[16 * w + k]);
            s4[k] += (double)h[16 * w + 8 + k];
        }
    }
    const char* names[8] = {"T Kblocks", "T epi+st", "g split0", "g K0", "g K1", "g K2", "g K3+y", "mix"};
    printf("per tile (cycles), %0.f tiles:\n", tiles);
    for (int k = 0; k < 8; ++k) printf("  %-10s wave0 %8.0f  wave4 %8.0f\n", names[k], s0[k] / tiles, s4[k] / tiles);
    return 0;
}
