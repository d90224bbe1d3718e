// train.h — kernels of the training step (csrc/train.hip): train-mode
// BatchNorm statistics and backward, the graph mix and its gradients, the
// weight-gradient GEMM (fp32 MFMA, split over rows), im2col / zero-upsample
// for the temporal-conv backward, the head's LeakyReLU + dropout, the MSE
// loss and Adam. The data-parallel GEMMs of the forward and of every input
// gradient run on the fp32 implicit-GEMM kernel (cgemm.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace tik {

// per-column partial sums over row chunks, double: part[chunk][c][2]
//   G == nullptr: (sum A, sum A^2)
//   G != nullptr: (sum G, sum G * (A - mean[c]))   (mean may be null -> 0)
// rows of C floats (ld = C). Returns the chunk count through *nchunk.
// M (optional, G mode): ReLU backward folded in, g = M > 0 ? G : 0.
hipError_t launch_colstats(const float* A, const float* G, const float* mean, long long R, int C, double* part,
                           int max_chunks, int* nchunk, hipStream_t st, const float* M = nullptr);
// train-mode BatchNorm statistics from colstats(A): mean, invstd, scale =
// gamma*invstd, shift = beta - mean*scale per column into stat[4][C]; running
// stats updated (momentum, unbiased variance). cmap: column -> channel
// (-1 = padding column: zero scale/shift), null = identity.
hipError_t launch_bn_fwd_finalize(const double* part, int nchunk, long long R, int C, const int* cmap,
                                  const float* gamma, const float* beta, float* run_mean, float* run_var,
                                  float momentum, float eps, float* stat, hipStream_t st);
// BatchNorm backward from colstats(G, A=x, mean): dgamma, dbeta (indexed by
// channel) and k[3][C] with dx = g*k0 + (x - mean)*k1 + k2.
hipError_t launch_bn_bwd_finalize(const double* part, int nchunk, long long R, int C, const int* cmap,
                                  const float* gamma, const float* stat, float* dgamma, float* dbeta, float* k,
                                  hipStream_t st);
// dst[c] = sum of the chunk partials' first sums (bias gradients)
hipError_t launch_colsum_finalize(const double* part, int nchunk, int C, float* dst, hipStream_t st);
// out = act(X*sc + sh + res), res = R2*sc2 + sh2 (sc2 != null), R2 (identity) or 0; rows of C floats
hipError_t launch_affine(float* out, const float* X, const float* sc, const float* sh, const float* R2,
                         const float* sc2, const float* sh2, long long R, int C, int relu, hipStream_t st);
// out = g*k0 + (x - mean)*k1 + k2 (BatchNorm input gradient); stat = bn_fwd_finalize's stat
// M (optional): g = M > 0 ? G : 0 (ReLU backward folded in)
hipError_t launch_bn_bwd_apply(float* out, const float* G, const float* X, const float* stat, const float* k,
                               long long R, int C, hipStream_t st, const float* M = nullptr);
// out = M > 0 ? G : 0 (ReLU backward on its output); n elements
hipError_t launch_relu_bwd(float* out, const float* G, const float* M, long long n, hipStream_t st);
// out[f][w][c] = sum_v Amat(v, w) in[f][v][c]; Amat = A (trans=0) or A^T (trans=1), V = 17
hipError_t launch_mix(float* out, const float* in, const float* A, int trans, long long frames, int C, hipStream_t st);
// dE[v][w] = A[v][w] * sum_{f,c} Y[f][v][c] dZ[f][w][c]  (edge-importance gradient), part: workspace
hipError_t launch_mix_grad(const float* Y, const float* dZ, long long frames, int C, const float* A, float* dE,
                           double* part, int max_chunks, hipStream_t st);
// C[m][n] = sum_r A[r][m] B[r][n] (weight gradients), fp32 MFMA, rows split
// over workgroups with deterministic partial sums in `part` (>= splits*M*N).
// Tap mode (taps.C > 0): B is a temporal conv's input (rows (nw*tin + t)*V + v
// of C floats, C % 64 == 0), read through the conv's row map (implicit
// im2col, N = kt*C), and C[m][ci*kt + tap] receives the torch weight layout.
struct WgradTaps {
    int C = 0, kt = 1, s = 1, pad = 0, tin = 1, tout = 1, V = 1;
};
hipError_t launch_wgrad(const float* A, int lda, const float* B, int ldb, int M, int N, long long R, float* C,
                        int ldc, float* part, long long part_cap, hipStream_t st, const WgradTaps& taps = WgradTaps());
// col[r][ci*kt + tap] = src[(n*tin + s*t + tap - pad)*V + v][ci] (0 outside the window)
hipError_t launch_im2col(float* col, const float* src, int lds, int C, int kt, int s, int pad, int N, int tin,
                         int tout, int V, hipStream_t st);
// up[(n*tin + t)*V + v][c] = t % s == 0 ? src[(n*tout + t/s)*V + v][c] : 0
hipError_t launch_upsample(float* up, const float* src, int C, int s, int N, int tin, int tout, int V, hipStream_t st);
// dst[i0*ds0 + i1*ds1 + i2*ds2] = src[soff + i0*ss0 + i1*ss1 + i2*ss2] (weight repacking)
hipError_t launch_permute(float* dst, const float* src, int d0, int d1, int d2, long long ds0, long long ds1,
                          long long ds2, long long soff, long long ss0, long long ss1, long long ss2, hipStream_t st);
// A batch of re-layouts in one launch: dst[i0*ds0 + i1*ds1 + i2*ds2] =
// src[s] (* src2[s] when src2 != null), s = soff + i0*ss0 + i1*ss1 + i2*ss2.
struct PermDesc {
    float* dst;
    const float* src;
    const float* src2;
    int d0, d1, d2;
    long long ds0, ds1, ds2, soff, ss0, ss1, ss2;
    long long block0;   // first workgroup (permute_batch_blocks)
};
// assigns block ranges; returns the grid size
long long permute_batch_blocks(PermDesc* descs, int nd);
hipError_t launch_permute_batch(const PermDesc* descs_dev, int nd, long long blocks, hipStream_t st);
// dst = a * b elementwise (n)
hipError_t launch_mul(float* dst, const float* a, const float* b, int n, hipStream_t st);
// dropout keep mask (1 with probability keep, else 0) from a counter-based hash of (seed, i)
hipError_t launch_dropout_mask(float* mask, long long n, float keep, unsigned long long seed, hipStream_t st);
// D = LeakyReLU(P, 0.01) * mask * scale
hipError_t launch_leaky_dropout(float* D, const float* P, const float* mask, float scale, long long n, hipStream_t st);
// dP = dD * mask * scale * (P > 0 ? 1 : 0.01)   (in place allowed: dP == dD)
hipError_t launch_leaky_dropout_bwd(float* dP, const float* dD, const float* P, const float* mask, float scale,
                                    long long n, hipStream_t st);
// MSE (nn.MSELoss, mean): loss[0] = mean((O - T)^2); dO = 2 (O - T) / n. O rows of ldo, T rows of
// cols floats, dO rows of ldo (padding columns zeroed)
hipError_t launch_mse(const float* O, int ldo, const float* T, long long rows, int cols, float* dO, float* loss,
                      hipStream_t st);
// torch.optim.Adam (single-tensor path): m = lerp(m, g, 1-b1); v = v*b2 + (1-b2) g^2;
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
hipError_t launch_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float b1, float b2,
                       float eps, double bc1, double bc2, hipStream_t st);

}  // namespace tik
