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
#include <algorithm>
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
                              "dbg128x128_DMA", "dbg128x128_MFMA", "dbg128x64_DMA", "dbg128x64_MFMA", "T128x128_W8", "T128x64_W8", "dbgW8_DMA", "dbgW8_MFMA"};
    return c < tik::C3_NCFG ? n[c] : "?";
}

// per-workgroup phase trace (s_memrealtime, 100 MHz): main loop vs epilogue
static void trace_launch(const char* tag, tik::Cgemm3Args a, int cfg, hipStream_t st, int nblocks) {
    unsigned long long* d;
    CK(hipMalloc(&d, (size_t)nblocks * 5 * 8));
    a.trace = d;
    for (int i = 0; i < 2; ++i) CK(tik::launch_cgemm3(a, cfg, st));
    CK(hipStreamSynchronize(st));
    std::vector<unsigned long long> h((size_t)nblocks * 5);
    CK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    CK(hipFree(d));
    unsigned long long t0 = ~0ull, t2 = 0;
    double loop = 0, epi = 0, wv = 0, wb = 0, wl = 0;
    for (int b = 0; b < nblocks; ++b) {
        const unsigned long long* t = &h[(size_t)b * 5];
        t0 = std::min(t0, t[0]); t2 = std::max(t2, t[2]);
        loop += (double)(t[1] - t[0]); epi += (double)(t[2] - t[1]);
        wv += (double)t[3]; wb += (double)(t[4] & 0xffffffffull); wl += (double)(t[4] >> 32);
    }
    const double span = (double)(t2 - t0);
    printf("  trace %-14s blocks %6d  span %8.1f us  loop %6.2f us  epilogue %6.2f us  resident/CU %.2f | wave0 loop %6.0f clk vm-wait %6.0f barrier %6.0f\n",
           tag, nblocks, span / 100.0, loop / nblocks / 100.0, epi / nblocks / 100.0, (loop + epi) / span / 256.0,
           wl / nblocks, wv / nblocks, wb / nblocks);
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
    const L layers[8] = {{4, 64, 1}, {64, 64, 1}, {64, 128, 2}, {128, 128, 1},
                         {128, 128, 1}, {128, 128, 2}, {128, 256, 2}, {256, 256, 2}};
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const size_t maxrows = (size_t)N * T0 * V;
    half_t* x = dev_halves(maxrows * 256 * 2, 1);   // SB rows (layer 0: one 32-channel block)
    half_t* z = dev_halves(maxrows * 256 * 2, 2);
    half_t* o = dev_halves(maxrows * 256 * 2, 3);
    half_t* wsb = dev_halves(256 * 3 * 8 * 64, 4);   // SB weights, up to Nc=256, kt=3, 8 blocks
    half_t* zeros;
    CK(hipMalloc(&zeros, 256));
    CK(hipMemset(zeros, 0, 256));
    float* bias = dev_floats(V * 256, 0.01f);
    float* amix = dev_floats(V * V, 0.05f);
    int tin = T0;
    double tot_best = 0, tot_cur = 0;
    const int only = argc > 4 ? atoi(argv[4]) : -1;   // profile one layer only
    for (int l = 0; l < 8; ++l) {
        const L& Ly = layers[l];
        if (only >= 0 && l != only) {
            tin = (tin - 1) / Ly.stride + 1;
            continue;
        }
        const int to = (tin - 1) / Ly.stride + 1;
        const long long rin = (long long)N * tin * V, rout = (long long)N * to * V;
        tik::Cgemm3Args g{};
        g.M = (int)rin; g.Nc = Ly.cout; g.V = V; g.tout = tin;
        const int nbi = tik::sb_blocks(Ly.cin), nbo = tik::sb_blocks(Ly.cout);
        g.seg[0] = tik::Seg3{x, nbi, 64 * nbi, 1, 1, 0, tin, wsb, 64 * nbi};
        g.nseg = 1; g.bias = bias; g.out_h = z; g.ldo = 64 * nbo; g.amix = amix;
        g.act = 1; g.mix_sparse = 1; g.zeros = zeros;
        const int gc[] = {tik::C3_G272x64, tik::C3_G272x128_W8};
        for (int f : {0, 1}) {
            g.tune = f;
            printf("L%d G %-12s %8.4f ms  flags %d\n", l, cfg_name(Ly.cout % 128 ? tik::C3_G272x64 : tik::C3_G272x128_W8),
                   time_launch(g, Ly.cout % 128 ? tik::C3_G272x64 : tik::C3_G272x128_W8, st, reps), f);
        }
        g.tune = 0;
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
        t.seg[0] = tik::Seg3{z, nbo, 64 * nbo, 3, Ly.stride, 1, tin, wsb, 3 * 64 * nbo};
        t.nseg = 1;
        if (Ly.cin != Ly.cout || Ly.stride != 1) {
            t.seg[1] = tik::Seg3{x, nbi, 64 * nbi, 1, Ly.stride, 0, tin, wsb, 64 * nbi};
            t.nseg = 2;
        } else {
            t.resid = x; t.ldr = 64 * nbi;
        }
        t.bias = bias; t.out_h = o; t.ldo = 64 * nbo; t.act = 1; t.zeros = zeros;
        const double tfl = 2.0 * rout * Ly.cout * (3.0 * Ly.cout + (t.nseg > 1 ? Ly.cin : 0));
        for (int f : {0, 1}) {
            t.tune = f;
            printf("L%d T %-12s %8.4f ms  flags %d\n", l, cfg_name(Ly.cout >= 128 ? tik::C3_T128x128 : tik::C3_T128x64),
                   time_launch(t, Ly.cout >= 128 ? tik::C3_T128x128 : tik::C3_T128x64, st, reps), f);
        }
        t.tune = 0;
        if (tik::tconv_halo_ok(t)) {
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            const int bn = Ly.cout >= 128 ? 128 : 64;
            for (int i = 0; i < 3; ++i) CK(tik::launch_tconv_halo(t, bn, st));
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < reps; ++i) CK(tik::launch_tconv_halo(t, bn, st));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("L%d T halo%-8d %8.4f ms  %6.1f TF(fp32-eq)\n", l, bn, ms / reps,
                   2.0 * rout * Ly.cout * (3.0 * Ly.cout + (t.nseg > 1 ? Ly.cin : 0)) / (ms / reps) / 1e9);
            // phase trace
            unsigned long long* d;
            const int nb = (int)((rout + 127) / 128) * (Ly.cout / bn);
            CK(hipMalloc(&d, (size_t)nb * 40));
            tik::Cgemm3Args tt = t;
            tt.trace = d;
            CK(tik::launch_tconv_halo(tt, bn, st));
            CK(hipStreamSynchronize(st));
            std::vector<unsigned long long> h((size_t)nb * 5);
            CK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
            CK(hipFree(d));
            double lp = 0, ep = 0, wv = 0, wb = 0, wl = 0;
            for (int b = 0; b < nb; ++b) {
                lp += (double)(h[5 * b + 1] - h[5 * b]); ep += (double)(h[5 * b + 2] - h[5 * b + 1]);
                wv += (double)h[5 * b + 3]; wb += (double)(h[5 * b + 4] & 0xffffffffull); wl += (double)(h[5 * b + 4] >> 32);
            }
            printf("  trace halo                                  loop %6.2f us  epilogue %6.2f us                  | wave0 loop %6.0f clk vm-wait %6.0f barrier %6.0f\n",
                   lp / nb / 100.0, ep / nb / 100.0, wl / nb, wv / nb, wb / nb);
        }
        {
            const int tg[] = {tik::TG_128x128, tik::TG_128x64, tik::TG_128x128_A4, tik::TG_128x64_A4};
            const char* tn[] = {"TG_128x128", "TG_128x64", "TG_128x128_A4", "TG_128x64_A4"};
            for (int q = 0; q < 4; ++q) {
                if (Ly.cout < 128 && (q == 0 || q == 2)) continue;
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                for (int i = 0; i < 3; ++i) CK(tik::launch_tgemm(t, tg[q], st));
                CK(hipEventRecord(e0, st));
                for (int i = 0; i < reps; ++i) CK(tik::launch_tgemm(t, tg[q], st));
                CK(hipEventRecord(e1, st));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf("L%d T %-12s %8.4f ms  %6.1f TF(fp32-eq)\n", l, tn[q], ms / reps,
                       2.0 * rout * Ly.cout * (3.0 * Ly.cout + (t.nseg > 1 ? Ly.cin : 0)) / (ms / reps) / 1e9);
            }
        }
        std::vector<int> tc;
        if (Ly.cout >= 128) tc = {tik::C3_T128x128, tik::C3_T128x128_W8, tik::C3_DBG_W8_DMA, tik::C3_DBG_W8_MFMA};
        else tc = {tik::C3_T128x64, tik::C3_T128x64_W8};
        best = 1e9; cur = 0;
        for (int c : tc) {
            const float ms = time_launch(t, c, st, reps);
            if (c == tc[0]) cur = ms;
            if (ms < best && (c < tik::C3_DBG_T128x128_DMA || c > tik::C3_DBG_T128x64_MFMA) && c < tik::C3_DBG_W8_DMA) best = ms;
            printf("L%d T %-12s %8.4f ms  %6.1f TF(fp32-eq)\n", l, cfg_name(c), ms, tfl / ms / 1e9);
        }
        tot_best += best; tot_cur += cur;
        {
            const int cfgT = Ly.cout >= 128 ? tik::C3_T128x128_W8 : tik::C3_T128x64_W8;
            const int nb = (int)((rout + 127) / 128) * (Ly.cout >= 128 ? (Ly.cout + 127) / 128 : (Ly.cout + 63) / 64);
            t.tune = 0;
            trace_launch(cfg_name(cfgT), t, cfgT, st, nb);
            const int cfgG = Ly.cout % 128 ? tik::C3_G272x64 : tik::C3_G272x128_W8;
            const int nbg = (int)((rin + 271) / 272) * (Ly.cout % 128 ? Ly.cout / 64 : Ly.cout / 128);
            g.tune = 0;
            trace_launch(cfg_name(cfgG), g, cfgG, st, nbg);
        }
        tin = to;
    }
    printf("backbone G+T: current configs %.4f ms, best-per-launch %.4f ms\n", tot_cur, tot_best);
    return 0;
}
