// train.hip — kernels of the training step (see train.h and trainer.cpp).
//
// Replaces the autograd graph of IKPoseTrainer.training_step
// (pose_trainer.py:146-155) and torch.optim.Adam (configure_optimizers,
// pose_trainer.py:196-197): BatchNorm in training mode (batch statistics,
// running-stat momentum update, st_gcn_aaai18.py:74-75,178,186,203), the
// graph-mix einsum and its gradients (gconv_origin.py:64 with the learnable
// edge importance, st_gcn_aaai18.py:104-108,129), ReLU / LeakyReLU / dropout
// backward, nn.MSELoss (pose_trainer.py:46-49) and the Adam update.
//
// Layout: activations are channels-last rows r = (n*T + t)*17 + v of C fp32.
// The per-channel reductions (BatchNorm statistics, bias and BN-parameter
// gradients) are column reductions over those rows: 64 consecutive columns
// per workgroup (coalesced 256-B row segments), rows split over chunks,
// double partial sums reduced in a fixed order (run-to-run deterministic).
#include <cstdlib>

#include "train.h"

namespace tik {

typedef float f32x4 __attribute__((ext_vector_type(4)));

static inline unsigned nblk(long long n, int b) { return (unsigned)((n + b - 1) / b); }

// ---------------------------------------------------------------- column statistics
// Workgroup = 16 column quads (64 columns, float4 loads: one 256-B row
// segment per 16 lanes) x 16 row lanes over a chunk of rows; double
// accumulators; the 16 row lanes reduced through LDS in a fixed order.
constexpr int CS_ROWS = 128;   // rows per chunk
__global__ __launch_bounds__(256) void colstats_kernel(const float* __restrict__ A, const float* __restrict__ G,
                                                       const float* __restrict__ M, const float* __restrict__ mean,
                                                       long long R, int C, long long rows_per,
                                                       double* __restrict__ part) {
    __shared__ double red[2][16][64];
    const int tid = threadIdx.x, q = tid & 15, rl = tid >> 4;
    const int c = blockIdx.x * 64 + 4 * q;
    const long long r0 = (long long)blockIdx.y * rows_per;
    const long long r1 = r0 + rows_per < R ? r0 + rows_per : R;
    double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
    if (c < C) {
        f32x4 mu = {0.f, 0.f, 0.f, 0.f};
        if (G && mean) mu = *reinterpret_cast<const f32x4*>(mean + c);
        for (long long r = r0 + rl; r < r1; r += 16) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(A + r * C + c);
            if (G) {
                f32x4 g = *reinterpret_cast<const f32x4*>(G + r * C + c);
                if (M) {   // ReLU backward folded in: g where the ReLU output is positive
                    const f32x4 mk = *reinterpret_cast<const f32x4*>(M + r * C + c);
#pragma unroll
                    for (int e = 0; e < 4; ++e) g[e] = mk[e] > 0.f ? g[e] : 0.f;
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    s1[e] += g[e];
                    s2[e] += (double)g[e] * (double)(a[e] - mu[e]);
                }
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    s1[e] += a[e];
                    s2[e] += (double)a[e] * a[e];
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        red[0][rl][4 * q + e] = s1[e];
        red[1][rl][4 * q + e] = s2[e];
    }
    __syncthreads();
    if (tid < 128) {
        const int k = tid >> 6, cl = tid & 63;
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < 16; ++i) t += red[k][i][cl];
        const int col = blockIdx.x * 64 + cl;
        if (col < C) part[((size_t)blockIdx.y * C + col) * 2 + k] = t;
    }
}

hipError_t launch_colstats(const float* A, const float* G, const float* mean, long long R, int C, double* part,
                           int max_chunks, int* nchunk, hipStream_t st, const float* M) {
    if (C % 4) return hipErrorInvalidValue;
    const int gx = (C + 63) / 64;
    constexpr int cs_rows = CS_ROWS;   // 128 measured best (256 -5 %, 64 +-0.3 %: profiles/r02_t15_train_ab.txt)
    long long nc = (R + cs_rows - 1) / cs_rows;
    if (nc > max_chunks) nc = max_chunks;
    if (nc < 1) nc = 1;
    const long long rows_per = R > 0 ? (R + nc - 1) / nc : 1;
    nc = R > 0 ? (R + rows_per - 1) / rows_per : 1;
    *nchunk = (int)nc;
    hipLaunchKernelGGL(colstats_kernel, dim3(gx, (unsigned)nc), dim3(256), 0, st, A, G, M, mean, R, C, rows_per, part);
    return hipGetLastError();
}

// sum over chunks of part[z][c][k] for one column: the 64 lanes of a wave
// stride the chunks, then a fixed xor-shuffle tree across the wave
__device__ __forceinline__ double chunk_sum64(const double* __restrict__ part, int nchunk, int C, int c, int k,
                                              int lane) {
    double s = 0.0;
    for (int z = lane; z < nchunk; z += 64) s += part[((size_t)z * C + c) * 2 + k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return s;
}

// finalize kernels: 256 threads = 4 columns, one wave (64 chunk lanes) each
__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const double* __restrict__ part, int nchunk, long long R,
                                                              int C, const int* __restrict__ cmap,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* run_mean,
                                                              float* run_var, float momentum, float eps,
                                                              float* __restrict__ stat) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= C) return;
    const double s1 = chunk_sum64(part, nchunk, C, c, 0, lane);
    const double s2 = chunk_sum64(part, nchunk, C, c, 1, lane);
    if (lane) return;
    const int p = cmap ? cmap[c] : c;
    if (p < 0) {
        stat[c] = 0.f; stat[C + c] = 0.f; stat[2 * C + c] = 0.f; stat[3 * C + c] = 0.f;
        return;
    }
    const double mean = s1 / (double)R;
    double var = s2 / (double)R - mean * mean;
    if (var < 0.0) var = 0.0;
    const float is = (float)(1.0 / sqrt(var + (double)eps));
    const float m = (float)mean;
    const float sc = gamma[p] * is;
    stat[c] = m;
    stat[C + c] = is;
    stat[2 * C + c] = sc;
    stat[3 * C + c] = beta[p] - m * sc;
    if (run_mean) {
        const double unb = R > 1 ? var * (double)R / (double)(R - 1) : var;
        run_mean[p] = (1.f - momentum) * run_mean[p] + momentum * m;
        run_var[p] = (1.f - momentum) * run_var[p] + momentum * (float)unb;
    }
}

hipError_t launch_bn_fwd_finalize(const double* part, int nchunk, long long R, int C, const int* cmap,
                                  const float* gamma, const float* beta, float* run_mean, float* run_var,
                                  float momentum, float eps, float* stat, hipStream_t st) {
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(nblk(C, 4)), dim3(256), 0, st, part, nchunk, R, C, cmap, gamma,
                       beta, run_mean, run_var, momentum, eps, stat);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* __restrict__ part, int nchunk, long long R,
                                                              int C, const int* __restrict__ cmap,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ stat, float* dgamma,
                                                              float* dbeta, float* __restrict__ k) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= C) return;
    const double s1 = chunk_sum64(part, nchunk, C, c, 0, lane);
    const double s2 = chunk_sum64(part, nchunk, C, c, 1, lane);
    if (lane) return;
    const int p = cmap ? cmap[c] : c;
    if (p < 0) {
        k[c] = 0.f; k[C + c] = 0.f; k[2 * C + c] = 0.f;
        return;
    }
    const double is = stat[C + c];
    const double g = gamma[p];
    dgamma[p] = (float)(s2 * is);
    dbeta[p] = (float)s1;
    // dx = g*is*(dy - mean(dy) - xhat*mean(dy*xhat))
    k[c] = (float)(g * is);
    k[C + c] = (float)(-g * is * is * is * s2 / (double)R);
    k[2 * C + c] = (float)(-g * is * s1 / (double)R);
}

hipError_t launch_bn_bwd_finalize(const double* part, int nchunk, long long R, int C, const int* cmap,
                                  const float* gamma, const float* stat, float* dgamma, float* dbeta, float* k,
                                  hipStream_t st) {
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(nblk(C, 4)), dim3(256), 0, st, part, nchunk, R, C, cmap, gamma,
                       stat, dgamma, dbeta, k);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void colsum_finalize_kernel(const double* __restrict__ part, int nchunk, int C,
                                                              float* dst) {
    const int lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= C) return;
    const double s = chunk_sum64(part, nchunk, C, c, 0, lane);
    if (lane == 0) dst[c] = (float)s;
}

hipError_t launch_colsum_finalize(const double* part, int nchunk, int C, float* dst, hipStream_t st) {
    hipLaunchKernelGGL(colsum_finalize_kernel, dim3(nblk(C, 4)), dim3(256), 0, st, part, nchunk, C, dst);
    return hipGetLastError();
}

// ---------------------------------------------------------------- elementwise
// float4 per thread (every C here is a multiple of 4); the channel index from
// 32-bit arithmetic (element counts stay below 2^31 in float4 units)
__global__ void affine_kernel(float* __restrict__ out, const float* __restrict__ X, const float* __restrict__ sc,
                              const float* __restrict__ sh, const float* __restrict__ R2,
                              const float* __restrict__ sc2, const float* __restrict__ sh2, unsigned n4, unsigned C4,
                              int relu) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const unsigned c = (i % C4) * 4;
    const f32x4 x = reinterpret_cast<const f32x4*>(X)[i];
    const f32x4 a = *reinterpret_cast<const f32x4*>(sc + c);
    const f32x4 b = *reinterpret_cast<const f32x4*>(sh + c);
    f32x4 v = x * a + b;
    if (R2) {
        const f32x4 r = reinterpret_cast<const f32x4*>(R2)[i];
        if (sc2) v += r * *reinterpret_cast<const f32x4*>(sc2 + c) + *reinterpret_cast<const f32x4*>(sh2 + c);
        else v += r;
    }
    if (relu)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
    reinterpret_cast<f32x4*>(out)[i] = v;
}

hipError_t launch_affine(float* out, const float* X, const float* sc, const float* sh, const float* R2,
                         const float* sc2, const float* sh2, long long R, int C, int relu, hipStream_t st) {
    const long long n = R * C;
    if (n == 0) return hipSuccess;
    if (C % 4 || n / 4 >= (1LL << 31)) return hipErrorInvalidValue;
    const unsigned n4 = (unsigned)(n / 4);
    hipLaunchKernelGGL(affine_kernel, dim3(nblk(n4, 256)), dim3(256), 0, st, out, X, sc, sh, R2, sc2, sh2, n4,
                       (unsigned)(C / 4), relu);
    return hipGetLastError();
}

__global__ void bn_bwd_apply_kernel(float* __restrict__ out, const float* __restrict__ G,
                                    const float* __restrict__ M, const float* __restrict__ X,
                                    const float* __restrict__ stat, const float* __restrict__ k, unsigned n4,
                                    unsigned C4) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const unsigned c = (i % C4) * 4, C = C4 * 4;
    f32x4 g = reinterpret_cast<const f32x4*>(G)[i];
    if (M) {
        const f32x4 m = reinterpret_cast<const f32x4*>(M)[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) g[e] = m[e] > 0.f ? g[e] : 0.f;
    }
    const f32x4 x = reinterpret_cast<const f32x4*>(X)[i];
    const f32x4 mu = *reinterpret_cast<const f32x4*>(stat + c);
    const f32x4 k0 = *reinterpret_cast<const f32x4*>(k + c);
    const f32x4 k1 = *reinterpret_cast<const f32x4*>(k + C + c);
    const f32x4 k2 = *reinterpret_cast<const f32x4*>(k + 2 * C + c);
    reinterpret_cast<f32x4*>(out)[i] = g * k0 + (x - mu) * k1 + k2;
}

hipError_t launch_bn_bwd_apply(float* out, const float* G, const float* X, const float* stat, const float* k,
                               long long R, int C, hipStream_t st, const float* M) {
    const long long n = R * C;
    if (n == 0) return hipSuccess;
    if (C % 4 || n / 4 >= (1LL << 31)) return hipErrorInvalidValue;
    const unsigned n4 = (unsigned)(n / 4);
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(nblk(n4, 256)), dim3(256), 0, st, out, G, M, X, stat, k, n4,
                       (unsigned)(C / 4));
    return hipGetLastError();
}

__global__ void relu_bwd_kernel(float* __restrict__ out, const float* __restrict__ G, const float* __restrict__ M,
                                long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = M[i] > 0.f ? G[i] : 0.f;
}

hipError_t launch_relu_bwd(float* out, const float* G, const float* M, long long n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(relu_bwd_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, out, G, M, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------- graph mix
// one thread per (frame, 4 channels): the 17 joint rows in registers, the
// 17x17 matrix in LDS (broadcast reads)
__global__ __launch_bounds__(256) void mix_kernel(float* __restrict__ out, const float* __restrict__ in,
                                                  const float* __restrict__ A, int trans, long long frames, int C) {
    __shared__ float As[17 * 17];
    for (int i = threadIdx.x; i < 289; i += 256) {
        const int v = i / 17, w = i % 17;
        As[i] = trans ? A[w * 17 + v] : A[i];
    }
    __syncthreads();
    const int C4 = C / 4;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= frames * C4) return;
    const long long f = idx / C4;
    const int c = (int)(idx % C4) * 4;
    const float* src = in + f * 17 * C + c;
    f32x4 y[17];
#pragma unroll
    for (int v = 0; v < 17; ++v) y[v] = *reinterpret_cast<const f32x4*>(src + (size_t)v * C);
    float* dst = out + f * 17 * C + c;
#pragma unroll
    for (int w = 0; w < 17; ++w) {
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int v = 0; v < 17; ++v) z += As[v * 17 + w] * y[v];
        *reinterpret_cast<f32x4*>(dst + (size_t)w * C) = z;
    }
}

hipError_t launch_mix(float* out, const float* in, const float* A, int trans, long long frames, int C, hipStream_t st) {
    if (C % 4) return hipErrorInvalidValue;
    const long long n = frames * (C / 4);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mix_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, out, in, A, trans, frames, C);
    return hipGetLastError();
}

// part[chunk][v*17 + w] = sum over the chunk's frames and all channels of
// Y[f][v][c] * dZ[f][w][c]: both 17 x C frame images staged in LDS (rows
// padded by one float), one (v, w) pair per thread (threads 0..32 take two)
constexpr int MIXG_CMAX = 256;
__global__ __launch_bounds__(256) void mix_grad_kernel(const float* __restrict__ Y, const float* __restrict__ G,
                                                       long long frames, int C, long long fpc,
                                                       double* __restrict__ part) {
    __shared__ float Ys[17 * (MIXG_CMAX + 1)];
    __shared__ float Gs[17 * (MIXG_CMAX + 1)];
    const int tid = threadIdx.x;
    const int ld = C + 1;
    const int p0 = tid, p1 = tid + 256;
    const int v0 = p0 / 17, w0 = p0 % 17;
    const int v1 = p1 / 17, w1 = p1 % 17;
    double acc0 = 0.0, acc1 = 0.0;
    const long long f0 = (long long)blockIdx.x * fpc;
    const long long f1 = f0 + fpc < frames ? f0 + fpc : frames;
    for (long long f = f0; f < f1; ++f) {
        const float* ys = Y + f * 17 * C;
        const float* gs = G + f * 17 * C;
        for (int i = tid; i < 17 * C; i += 256) {
            const int v = i / C, c = i - v * C;
            Ys[v * ld + c] = ys[i];
            Gs[v * ld + c] = gs[i];
        }
        __syncthreads();
        float s0 = 0.f, s1 = 0.f;
        for (int c = 0; c < C; ++c) {
            s0 += Ys[v0 * ld + c] * Gs[w0 * ld + c];
            if (p1 < 289) s1 += Ys[v1 * ld + c] * Gs[w1 * ld + c];
        }
        acc0 += s0;
        acc1 += s1;
        __syncthreads();
    }
    double* o = part + (size_t)blockIdx.x * 289;
    o[p0] = acc0;   // p0 < 256 < 289
    if (p1 < 289) o[p1] = acc1;
}

__global__ __launch_bounds__(256) void mix_grad_finalize_kernel(const double* __restrict__ part, int nchunk,
                                                                const float* __restrict__ A, float* dE) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per (v, w)
    if (i >= 289) return;
    double s = 0.0;
    for (int z = lane; z < nchunk; z += 64) s += part[(size_t)z * 289 + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) dE[i] = (float)s * A[i];
}

hipError_t launch_mix_grad(const float* Y, const float* dZ, long long frames, int C, const float* A, float* dE,
                           double* part, int max_chunks, hipStream_t st) {
    if (C > MIXG_CMAX) return hipErrorInvalidValue;
    long long nc = frames < 512 ? frames : 512;
    if (nc > max_chunks) nc = max_chunks;
    if (nc < 1) nc = 1;
    const long long fpc = (frames + nc - 1) / nc;
    nc = frames > 0 ? (frames + fpc - 1) / fpc : 0;
    if (nc > 0)
        hipLaunchKernelGGL(mix_grad_kernel, dim3((unsigned)nc), dim3(256), 0, st, Y, dZ, frames, C, fpc, part);
    hipLaunchKernelGGL(mix_grad_finalize_kernel, dim3(nblk(289, 4)), dim3(256), 0, st, part, (int)nc, A, dE);
    return hipGetLastError();
}

// ---------------------------------------------------------------- weight-gradient GEMM
// C[m][n] = sum_r A[r][m] B[r][n]: 64 x 64 output tile per workgroup, 4 waves
// of 32 x 32 (2 x 2 v_mfma_f32_16x16x4_f32 fragments), 16 rows per LDS step
// (A and B staged [row][64 + 16 pad] so a 16-lane group reads 16 consecutive
// floats of one row and the four groups land on distinct banks). MFMA
// operands: A-op lane l = A^T[m = l&15][k = l>>4] = As[k][m], B-op =
// Bs[k][n]; D lane l holds rows 4(l>>4)+e, column l&15.
// Tap mode (g.C > 0): B is the conv input itself, read through the temporal
// conv's row map (implicit im2col): column n = tap*C + ci of row r is
// B[(nw*tin + s*t + tap - pad)*V + v][ci] (zero outside the window), r =
// (nw*tout + t)*V + v; a 64-column tile never straddles taps (C % 64 == 0).
__global__ __launch_bounds__(256) void wgrad_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                    int ldb, int M, int N, long long R, long long rows_per,
                                                    float* __restrict__ part, WgradTaps g) {
    constexpr int LDS_LD = 80;
    __shared__ float As[16 * LDS_LD];
    __shared__ float Bs[16 * LDS_LD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
    const long long r0 = (long long)blockIdx.z * rows_per;
    const long long r1 = r0 + rows_per < R ? r0 + rows_per : R;
    const int lr = tid >> 4, c4 = (tid & 15) * 4;
    const bool avec = (lda % 4 == 0) && (m0 + c4 + 3 < M);
    const bool bvec = (ldb % 4 == 0) && (n0 + c4 + 3 < N);
    const int tap = g.C ? n0 / g.C : 0;
    const int bcol = g.C ? n0 - tap * g.C : n0;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // tap mode: this thread's row r0 + lr decoded once into (window, frame,
    // joint), then advanced incrementally by 16 rows per step (V = 17 > 16:
    // at most one joint wrap and one frame wrap per step; no 64-bit divides
    // in the loop)
    int tv = 0, tt = 0;
    long long tn = 0;
    if (g.C) {
        const long long row = r0 + lr;
        tv = (int)(row % g.V);
        const long long q = row / g.V;
        tt = (int)(q % g.tout);
        tn = q / g.tout;
    }
    // rows r .. r+15 of A and B into registers (zero past the chunk / matrix edge)
    auto load = [&](long long r, f32x4& av, f32x4& bv) {
        av = f32x4{0.f, 0.f, 0.f, 0.f};
        bv = f32x4{0.f, 0.f, 0.f, 0.f};
        const long long row = r + lr;
        long long brow = row;
        bool bok = true;
        if (g.C) {
            const int ts = g.s * tt + tap - g.pad;
            bok = ts >= 0 && ts < g.tin;
            brow = (tn * g.tin + ts) * g.V + tv;
            tv += 16;
            if (tv >= g.V) {
                tv -= g.V;
                if (++tt >= g.tout) { tt = 0; ++tn; }
            }
        }
        if (row < r1) {
            const float* ap = A + row * lda + m0 + c4;
            const float* bp = B + brow * ldb + bcol + c4;
            if (avec) av = *reinterpret_cast<const f32x4*>(ap);
            else
                for (int e = 0; e < 4; ++e) av[e] = (m0 + c4 + e < M) ? ap[e] : 0.f;
            if (!bok) {
            } else if (bvec) {
                bv = *reinterpret_cast<const f32x4*>(bp);
            } else {
                for (int e = 0; e < 4; ++e) bv[e] = (n0 + c4 + e < N) ? bp[e] : 0.f;
            }
        }
    };
    f32x4 av, bv;
    load(r0, av, bv);
    for (long long r = r0; r < r1; r += 16) {
        __syncthreads();
        *reinterpret_cast<f32x4*>(As + lr * LDS_LD + c4) = av;
        *reinterpret_cast<f32x4*>(Bs + lr * LDS_LD + c4) = bv;
        __syncthreads();
        // the next 16 rows' global loads are in flight during this step's MFMAs
        if (r + 16 < r1) load(r + 16, av, bv);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
            const int k = kk * 4 + (lane >> 4);
            float a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[k * LDS_LD + wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Bs[k * LDS_LD + wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    }
    float* o = part + (size_t)blockIdx.z * M * N;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + e;
                const int n = n0 + wn * 32 + j * 16 + (lane & 15);
                if (m < M && n < N) o[(size_t)m * N + n] = acc[i][j][e];
            }
}

// sum of the row-split partials; tap mode stores column tap*C + ci at ci*kt + tap
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int M, int N, float* C, int ldc,
                                    int tapC, int kt) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)M * N) return;
    const size_t st = (size_t)M * N;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int z = 0;
    for (; z + 3 < splits; z += 4) {
        s0 += part[(size_t)z * st + i];
        s1 += part[(size_t)(z + 1) * st + i];
        s2 += part[(size_t)(z + 2) * st + i];
        s3 += part[(size_t)(z + 3) * st + i];
    }
    for (; z < splits; ++z) s0 += part[(size_t)z * st + i];
    const int n = (int)(i % N);
    const int col = tapC ? (n % tapC) * kt + n / tapC : n;
    C[(i / N) * ldc + col] = (s0 + s1) + (s2 + s3);
}

hipError_t launch_wgrad(const float* A, int lda, const float* B, int ldb, int M, int N, long long R, float* C,
                        int ldc, float* part, long long part_cap, hipStream_t st, const WgradTaps& g) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (g.C && (g.C % 64 || N != g.kt * g.C || g.V <= 16 || g.tout <= 0)) return hipErrorInvalidValue;
    const int gx = (M + 63) / 64, gy = (N + 63) / 64;
    constexpr int target = 512;   // workgroups (256 -3 %, 1024 +-0.3 %: profiles/r02_t15_train_ab.txt)
    long long splits = target / (gx * gy);
    const long long max_by_rows = (R + 255) / 256;   // >= 256 rows per split
    if (splits > max_by_rows) splits = max_by_rows;
    if (splits > part_cap / ((long long)M * N)) splits = part_cap / ((long long)M * N);
    if (splits < 1) splits = 1;
    if ((long long)M * N > part_cap) return hipErrorInvalidValue;
    long long rows_per = (R + splits - 1) / splits;
    rows_per = (rows_per + 15) / 16 * 16;
    if (rows_per < 16) rows_per = 16;
    splits = R > 0 ? (R + rows_per - 1) / rows_per : 1;
    hipLaunchKernelGGL(wgrad_kernel, dim3(gx, gy, (unsigned)splits), dim3(256), 0, st, A, lda, B, ldb, M, N, R,
                       rows_per, part, g);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(nblk((long long)M * N, 256)), dim3(256), 0, st, part, (int)splits, M,
                       N, C, ldc, g.C, g.kt);
    return hipGetLastError();
}

// ---------------------------------------------------------------- temporal-conv helpers
__global__ void im2col_kernel(float* __restrict__ col, const float* __restrict__ src, int lds, int C, int kt, int s,
                              int pad, long long n_out, int tin, int tout, int V) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_out * C) return;
    const long long r = i / C;
    const int ci = (int)(i % C);
    const int v = (int)(r % V);
    const long long q = r / V;
    const int t = (int)(q % tout);
    const long long n = q / tout;
    float* o = col + r * ((long long)C * kt) + (long long)ci * kt;
    for (int tap = 0; tap < kt; ++tap) {
        const int ts = s * t + tap - pad;
        o[tap] = (ts >= 0 && ts < tin) ? src[((n * tin + ts) * V + v) * lds + ci] : 0.f;
    }
}

hipError_t launch_im2col(float* col, const float* src, int lds, int C, int kt, int s, int pad, int N, int tin,
                         int tout, int V, hipStream_t st) {
    const long long n_out = (long long)N * tout * V;
    if (n_out * C == 0) return hipSuccess;
    hipLaunchKernelGGL(im2col_kernel, dim3(nblk(n_out * C, 256)), dim3(256), 0, st, col, src, lds, C, kt, s, pad,
                       n_out, tin, tout, V);
    return hipGetLastError();
}

// float4 per thread, 32-bit index arithmetic (counts < 2^31 in float4 units)
__global__ void upsample_kernel(float* __restrict__ up, const float* __restrict__ src, unsigned C4, int s,
                                unsigned n4, unsigned tin, unsigned tout, unsigned V) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const unsigned r = i / C4, c4 = i - r * C4;
    const unsigned q = r / V, v = r - q * V;
    const unsigned n = q / tin, t = q - n * tin;
    f32x4 val = {0.f, 0.f, 0.f, 0.f};
    if (t % s == 0) val = reinterpret_cast<const f32x4*>(src)[((n * tout + t / s) * V + v) * C4 + c4];
    reinterpret_cast<f32x4*>(up)[i] = val;
}

hipError_t launch_upsample(float* up, const float* src, int C, int s, int N, int tin, int tout, int V, hipStream_t st) {
    const long long n_in = (long long)N * tin * V;
    if (n_in * C == 0) return hipSuccess;
    if (C % 4 || n_in * C / 4 >= (1LL << 31)) return hipErrorInvalidValue;
    const unsigned n4 = (unsigned)(n_in * C / 4);
    hipLaunchKernelGGL(upsample_kernel, dim3(nblk(n4, 256)), dim3(256), 0, st, up, src, (unsigned)(C / 4), s, n4,
                       (unsigned)tin, (unsigned)tout, (unsigned)V);
    return hipGetLastError();
}

__global__ void permute_kernel(float* __restrict__ dst, const float* __restrict__ src, int d0, int d1, int d2,
                               long long ds0, long long ds1, long long ds2, long long soff, long long ss0,
                               long long ss1, long long ss2) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)d0 * d1 * d2) return;
    const int i2 = (int)(i % d2);
    const long long q = i / d2;
    const int i1 = (int)(q % d1);
    const int i0 = (int)(q / d1);
    dst[i0 * ds0 + i1 * ds1 + i2 * ds2] = src[soff + i0 * ss0 + i1 * ss1 + i2 * ss2];
}

hipError_t launch_permute(float* dst, const float* src, int d0, int d1, int d2, long long ds0, long long ds1,
                          long long ds2, long long soff, long long ss0, long long ss1, long long ss2, hipStream_t st) {
    const long long n = (long long)d0 * d1 * d2;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(permute_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, dst, src, d0, d1, d2, ds0, ds1, ds2, soff,
                       ss0, ss1, ss2);
    return hipGetLastError();
}

// every weight re-layout of a step in one launch: workgroup b serves the
// descriptor whose block range holds b (ranges laid out by the host)
__global__ __launch_bounds__(256) void permute_batch_kernel(const PermDesc* __restrict__ descs, int nd) {
    int d = 0;
    while (d + 1 < nd && descs[d + 1].block0 <= (long long)blockIdx.x) ++d;
    const PermDesc& q = descs[d];
    const long long n = (long long)q.d0 * q.d1 * q.d2;
    for (long long i = (blockIdx.x - q.block0) * 1024LL + threadIdx.x, e = 0; e < 4; ++e, i += 256) {
        if (i >= n) return;
        const int i2 = (int)(i % q.d2);
        const long long r = i / q.d2;
        const int i1 = (int)(r % q.d1);
        const int i0 = (int)(r / q.d1);
        const long long so = q.soff + i0 * q.ss0 + i1 * q.ss1 + i2 * q.ss2;
        const float v = q.src[so];
        q.dst[i0 * q.ds0 + i1 * q.ds1 + i2 * q.ds2] = q.src2 ? v * q.src2[so] : v;
    }
}

long long permute_batch_blocks(PermDesc* descs, int nd) {
    long long b = 0;
    for (int d = 0; d < nd; ++d) {
        descs[d].block0 = b;
        b += ((long long)descs[d].d0 * descs[d].d1 * descs[d].d2 + 1023) / 1024;
    }
    return b;
}

hipError_t launch_permute_batch(const PermDesc* descs_dev, int nd, long long blocks, hipStream_t st) {
    if (nd == 0 || blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(permute_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, st, descs_dev, nd);
    return hipGetLastError();
}

__global__ void mul_kernel(float* dst, const float* a, const float* b, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = a[i] * b[i];
}

hipError_t launch_mul(float* dst, const float* a, const float* b, int n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mul_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, dst, a, b, n);
    return hipGetLastError();
}

// ---------------------------------------------------------------- head
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void dropout_mask_kernel(float* mask, long long n, float keep, unsigned long long seed) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long h = splitmix64(seed ^ splitmix64((unsigned long long)i));
    const float u = (float)(h >> 40) * (1.0f / 16777216.0f);   // 24-bit uniform in [0, 1)
    mask[i] = u < keep ? 1.f : 0.f;
}

hipError_t launch_dropout_mask(float* mask, long long n, float keep, unsigned long long seed, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(dropout_mask_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, mask, n, keep, seed);
    return hipGetLastError();
}

__global__ void leaky_dropout_kernel(float* __restrict__ D, const float* __restrict__ P, const float* __restrict__ mask,
                                     float scale, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float p = P[i];
    const float l = p > 0.f ? p : 0.01f * p;
    D[i] = l * (mask[i] * scale);
}

hipError_t launch_leaky_dropout(float* D, const float* P, const float* mask, float scale, long long n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(leaky_dropout_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, D, P, mask, scale, n);
    return hipGetLastError();
}

__global__ void leaky_dropout_bwd_kernel(float* dP, const float* dD, const float* __restrict__ P,
                                         const float* __restrict__ mask, float scale, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float g = dD[i] * (mask[i] * scale);
    dP[i] = P[i] > 0.f ? g : g * 0.01f;
}

hipError_t launch_leaky_dropout_bwd(float* dP, const float* dD, const float* P, const float* mask, float scale,
                                    long long n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(leaky_dropout_bwd_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, dP, dD, P, mask, scale, n);
    return hipGetLastError();
}

// one workgroup: the loss is a few thousand to a few hundred thousand elements
__global__ __launch_bounds__(1024) void mse_kernel(const float* __restrict__ O, int ldo, const float* __restrict__ T,
                                                   long long rows, int cols, float* __restrict__ dO,
                                                   float* __restrict__ loss) {
    __shared__ double red[1024];
    const long long n = rows * cols;
    const float inv = 2.f / (float)n;
    double s = 0.0;
    for (long long i = threadIdx.x; i < rows * ldo; i += blockDim.x) {
        const long long r = i / ldo;
        const int c = (int)(i % ldo);
        if (c < cols) {
            const float d = O[i] - T[r * cols + c];
            s += (double)d * d;
            dO[i] = inv * d;
        } else {
            dO[i] = 0.f;
        }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) loss[0] = (float)(red[0] / (double)n);
}

hipError_t launch_mse(const float* O, int ldo, const float* T, long long rows, int cols, float* dO, float* loss,
                      hipStream_t st) {
    hipLaunchKernelGGL(mse_kernel, dim3(1), dim3(1024), 0, st, O, ldo, T, rows, cols, dO, loss);
    return hipGetLastError();
}

// ---------------------------------------------------------------- Adam
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long long n, float w1, float b2, float w2, float step_size,
                            float bc2_sqrt, float eps) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float gi = g[i];
    float mi = m[i];
    mi = mi + w1 * (gi - mi);                 // exp_avg.lerp_(grad, 1 - beta1)
    float vi = v[i] * b2;                     // exp_avg_sq.mul_(beta2)
    vi = vi + w2 * gi * gi;                   //           .addcmul_(grad, grad, value=1 - beta2)
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + step_size * (mi / denom);   // param.addcdiv_(exp_avg, denom, value=-step_size)
    m[i] = mi;
    v[i] = vi;
}

hipError_t launch_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float b1, float b2,
                       float eps, double bc1, double bc2, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const float w1 = (float)(1.0 - (double)b1), w2 = (float)(1.0 - (double)b2);
    const float step_size = (float)(-(double)lr / bc1);
    const float bc2s = (float)sqrt(bc2);
    hipLaunchKernelGGL(adam_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, p, g, m, v, n, w1, b2, w2, step_size, bc2s,
                       eps);
    return hipGetLastError();
}

}  // namespace tik
