// lds_victim.hip — does anything else running on the GPU write into this
// workgroup's LDS? Each workgroup (256 threads, ~18 KB LDS like gcn0)
// fills its LDS with a pattern, then re-reads and checks it for a while,
// counting words that changed. Run beside other processes' kernels.
// MODE 0: each lane re-reads its own words; MODE 1: broadcast reads (every
// lane of a wave reads the same word); MODE 2 / 3: wave-uniform 16-B aligned
// ds_read_b128 / ds_read_b96 (how the pre-fix gcn0 read its mix constants).
//   lds_victim SECONDS [MODE]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int WORDS = 4640;   // 18,560 B
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v3u __attribute__((ext_vector_type(3)));

__global__ __launch_bounds__(256) void victim(unsigned seed, int iters, int mode, unsigned long long* bad, unsigned* first) {
    __shared__ __attribute__((aligned(16))) unsigned s[WORDS];
    const unsigned key = seed * 2654435761u + blockIdx.x * 40503u;
    for (int i = threadIdx.x; i < WORDS; i += 256) s[i] = key ^ (i * 0x9E3779B9u);
    __syncthreads();
    unsigned long long c = 0;
    for (int it = 0; it < iters; ++it) {
        for (int i0 = threadIdx.x; i0 < WORDS; i0 += 256) {
            if (mode <= 1) {
                // broadcast: the wave's lanes all read word (i0 - lane) (wave-uniform)
                const int i = mode ? __builtin_amdgcn_readfirstlane(i0) : i0;
                const unsigned v = s[i];
                if (v != (key ^ (i * 0x9E3779B9u))) {
                    ++c;
                    atomicCAS(first, 0xFFFFFFFFu, (unsigned)i);
                }
            } else {
                // wave-uniform 16-B aligned vector reads: ds_read_b128 (mode 2) or ds_read_b96 (mode 3)
                const int i = __builtin_amdgcn_readfirstlane(i0 & ~3) + 4 * ((threadIdx.x >> 6) & 1);
                if (i + 3 >= WORDS) continue;
                unsigned w[4];
                if (mode == 2) {
                    const v4u t = *reinterpret_cast<const v4u*>(s + i);
                    w[0] = t[0]; w[1] = t[1]; w[2] = t[2]; w[3] = t[3];
                } else {
                    const v3u t = *reinterpret_cast<const v3u*>(s + i);
                    w[0] = t[0]; w[1] = t[1]; w[2] = t[2]; w[3] = key ^ ((i + 3) * 0x9E3779B9u);
                }
                for (int e = 0; e < 4; ++e)
                    if (w[e] != (key ^ ((i + e) * 0x9E3779B9u))) {
                        ++c;
                        atomicCAS(first, 0xFFFFFFFFu, (unsigned)(i + e));
                    }
            }
        }
        __builtin_amdgcn_s_sleep(8);
    }
    if (c) atomicAdd(bad, c);
}

int main(int argc, char** argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 20.0;
    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    unsigned long long* bad;
    unsigned* first;
    CK(hipMalloc(&bad, 8));
    CK(hipMalloc(&first, 4));
    CK(hipMemset(bad, 0, 8));
    CK(hipMemset(first, 0xFF, 4));
    const auto t0 = std::chrono::steady_clock::now();
    unsigned seed = 1;
    int launches = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
        hipLaunchKernelGGL(victim, dim3(2048), dim3(256), 0, 0, seed++, 200, mode, bad, first);
        CK(hipDeviceSynchronize());
        ++launches;
    }
    unsigned long long hb = 0;
    unsigned hf = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost));
    printf("{\"mode\": %d, \"launches\": %d, \"bad_words\": %llu, \"first_bad_word\": %d}\n", mode, launches, hb, (int)hf);
    return 0;
}
