// lds_victim.hip — does anything else running on the GPU write into this
// workgroup's LDS? Each workgroup (256 threads, ~18 KB LDS like gcn0)
// fills its LDS with a pattern, then re-reads and checks it for a while,
// counting words that changed. Run beside other processes' kernels.
//   lds_victim SECONDS
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

__global__ __launch_bounds__(256) void victim(unsigned seed, int iters, unsigned long long* bad, unsigned* first) {
    __shared__ unsigned s[WORDS];
    const unsigned key = seed * 2654435761u + blockIdx.x * 40503u;
    for (int i = threadIdx.x; i < WORDS; i += 256) s[i] = key ^ (i * 0x9E3779B9u);
    __syncthreads();
    unsigned long long c = 0;
    for (int it = 0; it < iters; ++it) {
        for (int i = threadIdx.x; i < WORDS; i += 256) {
            const unsigned v = s[i];
            if (v != (key ^ (i * 0x9E3779B9u))) {
                ++c;
                atomicCAS(first, 0xFFFFFFFFu, (unsigned)i);
            }
        }
        __builtin_amdgcn_s_sleep(8);
    }
    if (c) atomicAdd(bad, c);
}

int main(int argc, char** argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 20.0;
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
        hipLaunchKernelGGL(victim, dim3(2048), dim3(256), 0, 0, seed++, 200, bad, first);
        CK(hipDeviceSynchronize());
        ++launches;
    }
    unsigned long long hb = 0;
    unsigned hf = 0;
    CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost));
    printf("{\"launches\": %d, \"bad_words\": %llu, \"first_bad_word\": %d}\n", launches, hb, (int)hf);
    return 0;
}
