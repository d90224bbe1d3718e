// misc.hip — the small (HBM/latency-bound) kernels of the IK path:
//   * data_bn on load            st_gcn_aaai18.py:119-125 (+ data_bn :74-75)
//   * angle-axis -> rotmat       common/kornia_geometry_conversion.py:125-201
//   * window gather              mmskeleton/datasets/data_amass.py:18-42, 221-236
//   * generic ConvTemporalGraphical (reference NCTV layout)  gconv_origin.py:56-65
#include "misc.h"
#include "online.h"

namespace tik {

// x (rows, V, C) -> xb (rows, V, 4): per-(v,c) eval BatchNorm1d over the
// (V*C) channels of the permuted input, channel index v*C + c
// (st_gcn_aaai18.py:120-122); 4th channel zero so the next GEMM reads float4.
__global__ void data_bn_kernel(const float* __restrict__ x, int n_px, int V, int C,
                               const float* __restrict__ scale, const float* __restrict__ shift,
                               float* __restrict__ xb) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;   // pixel = (frame, v)
    if (p >= n_px) return;
    const int v = p % V;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C && c < 4; ++c) {
        const int j = v * C + c;
        o[c] = fmaf(x[(size_t)p * C + c], scale[j], shift[j]);
    }
    reinterpret_cast<float4*>(xb)[p] = make_float4(o[0], o[1], o[2], o[3]);
}

hipError_t launch_data_bn(const float* x, int n_px, int V, int C, const float* scale,
                          const float* shift, float* xb, hipStream_t st) {
    if (n_px <= 0) return hipSuccess;
    (void)hipGetLastError();  // drop a stale error left by earlier runtime calls
    hipLaunchKernelGGL(data_bn_kernel, dim3((n_px + 255) / 256), dim3(256), 0, st, x, n_px, V, C,
                       scale, shift, xb);
    return hipGetLastError();
}

// kornia: theta2 = aa.aa; if theta2 > 1e-6: w = aa/(theta+1e-6), Rodrigues;
// else Taylor [1,-rz,ry; rz,1,-rx; -ry,rx,1].
__global__ void aa_to_rotmat_kernel(const float* __restrict__ aa, int n, float* __restrict__ R) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float rx = aa[3 * i], ry = aa[3 * i + 1], rz = aa[3 * i + 2];
    const float th2 = rx * rx + ry * ry + rz * rz;
    float m[9];
    if (th2 > 1e-6f) {
        const float th = sqrtf(th2);
        const float inv = 1.0f / (th + 1e-6f);
        const float wx = rx * inv, wy = ry * inv, wz = rz * inv;
        float s, c;
        sincosf(th, &s, &c);
        const float oc = 1.0f - c;
        m[0] = c + wx * wx * oc;       m[1] = wx * wy * oc - wz * s;  m[2] = wy * s + wx * wz * oc;
        m[3] = wz * s + wx * wy * oc;  m[4] = c + wy * wy * oc;       m[5] = -wx * s + wy * wz * oc;
        m[6] = -wy * s + wx * wz * oc; m[7] = wx * s + wy * wz * oc;  m[8] = c + wz * wz * oc;
    } else {
        m[0] = 1.f; m[1] = -rz; m[2] = ry;
        m[3] = rz;  m[4] = 1.f; m[5] = -rx;
        m[6] = -ry; m[7] = rx;  m[8] = 1.f;
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) R[9 * i + k] = m[k];
}

hipError_t launch_aa_to_rotmat(const float* aa, int n, float* R, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    (void)hipGetLastError();  // drop a stale error left by earlier runtime calls
    hipLaunchKernelGGL(aa_to_rotmat_kernel, dim3((n + 255) / 256), dim3(256), 0, st, aa, n, R);
    return hipGetLastError();
}

// windows[i][k][v][c] = seq[clamp(idx0+i-h+k)][v][c] - root(frame), one thread
// per (window, frame, joint); c = 0..2.
__global__ void window_gather_kernel(const float* __restrict__ seq, int F, int V, int idx0, int n_idx,
                                     int h, int ra, int rb, int relative, float* __restrict__ out) {
    const int W = 2 * h + 1;
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total = (long long)n_idx * W * V;
    if (p >= total) return;
    const int v = (int)(p % V);
    const long long q = p / V;
    const int k = (int)(q % W);
    const int i = (int)(q / W);
    int t = idx0 + i - h + k;
    t = t < 0 ? 0 : (t >= F ? F - 1 : t);
    const float* fr = seq + (size_t)t * V * 3;
    float o0 = fr[v * 3], o1 = fr[v * 3 + 1], o2 = fr[v * 3 + 2];
    if (relative) {
        o0 -= 0.5f * (fr[ra * 3] + fr[rb * 3]);
        o1 -= 0.5f * (fr[ra * 3 + 1] + fr[rb * 3 + 1]);
        o2 -= 0.5f * (fr[ra * 3 + 2] + fr[rb * 3 + 2]);
    }
    out[p * 3] = o0;
    out[p * 3 + 1] = o1;
    out[p * 3 + 2] = o2;
}

hipError_t launch_window_gather(const float* seq, int F, int V, int idx0, int n_idx, int h, int ra,
                                int rb, int relative, float* out, hipStream_t st) {
    const long long total = (long long)n_idx * (2 * h + 1) * V;
    if (total <= 0) return hipSuccess;
    (void)hipGetLastError();  // drop a stale error left by earlier runtime calls
    hipLaunchKernelGGL(window_gather_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       seq, F, V, idx0, n_idx, h, ra, rb, relative, out);
    return hipGetLastError();
}

// Generic ConvTemporalGraphical (any K, V, t-kernel/stride/padding/dilation),
// reference layout: x (N,Cin,T,V), W (K*Cout,Cin,tk,1), out (N,Cout,To,V).
// Stage 1: y[n][k*Cout+c][to][v] = b + sum_{ci,j} W[..][ci][j] x[n][ci][to*s - p + j*d][v]
// Stage 2: out[n][c][to][w] = sum_{k,v} y[n][k*Cout+c][to][v] A[k][v][w]
// One block per (n, to); y for that frame lives in LDS (K*Cout*V floats).
__global__ void gconv_kernel(const float* __restrict__ x, int Cin, int T, int V,
                             const float* __restrict__ A, int K, const float* __restrict__ W,
                             const float* __restrict__ b, int Cout, int tk, int ts, int tp, int td,
                             int To, float* __restrict__ out) {
    extern __shared__ float ys[];   // [K*Cout][V]
    const int n = blockIdx.y, to = blockIdx.x;
    const int KC = K * Cout;
    for (int p = threadIdx.x; p < KC * V; p += blockDim.x) {
        const int o = p / V, v = p % V;
        float s = b ? b[o] : 0.f;
        for (int j = 0; j < tk; ++j) {
            const int t = to * ts - tp + j * td;
            if (t < 0 || t >= T) continue;
            for (int ci = 0; ci < Cin; ++ci)
                s = fmaf(W[((size_t)o * Cin + ci) * tk + j], x[(((size_t)n * Cin + ci) * T + t) * V + v], s);
        }
        ys[p] = s;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < Cout * V; p += blockDim.x) {
        const int c = p / V, w = p % V;
        float s = 0.f;
        for (int k = 0; k < K; ++k)
            for (int v = 0; v < V; ++v) s = fmaf(ys[(k * Cout + c) * V + v], A[((size_t)k * V + v) * V + w], s);
        out[(((size_t)n * Cout + c) * To + to) * V + w] = s;
    }
}

hipError_t launch_gconv(const float* x, int N, int Cin, int T, int V, const float* A, int K,
                        const float* W, const float* b, int Cout, int tk, int ts, int tp, int td,
                        int To, float* out, hipStream_t st) {
    if (N <= 0 || To <= 0) return hipSuccess;
    const size_t shm = (size_t)K * Cout * V * sizeof(float);
    if (shm > 160 * 1024) return hipErrorInvalidValue;
    if (shm > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gconv_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
        if (e != hipSuccess) return e;
    }
    (void)hipGetLastError();  // drop a stale error left by earlier runtime calls
    hipLaunchKernelGGL(gconv_kernel, dim3(To, N), dim3(256), shm, st, x, Cin, T, V, A, K, W, b, Cout,
                       tk, ts, tp, td, To, out);
    return hipGetLastError();
}

// Copy rows of C floats into rows of Cp >= C floats, zero-filling the tail.
__global__ void pad_channels_kernel(const float* __restrict__ x, long long rows, int C, int Cp,
                                    float* __restrict__ y) {
    const long long p = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= rows * Cp) return;
    const long long r = p / Cp;
    const int c = (int)(p - r * Cp);
    y[p] = c < C ? x[r * C + c] : 0.f;
}

hipError_t launch_pad_channels(const float* x, long long rows, int C, int Cp, float* y, hipStream_t st) {
    const long long total = rows * Cp;
    if (total <= 0) return hipSuccess;
    (void)hipGetLastError();  // drop a stale error left by earlier runtime calls
    hipLaunchKernelGGL(pad_channels_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, x,
                       rows, C, Cp, y);
    return hipGetLastError();
}

// ---- online (streaming) windowing: device ring of the last W = 2h+1 frames.
// push: ring[count % W] = frame; ++count.  (one block)
__global__ void stream_push_kernel(float* ring, int W, int nv, int* count, const float* frame) {
    const int c = *count;
    float* slot = ring + (size_t)(c % W) * nv;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) slot[i] = frame[i];
    __syncthreads();
    if (threadIdx.x == 0) *count = stream_next_count(c, W);
}

// window centred at c = count-1-h: frames c-h .. c+h = count-1-2h .. count-1,
// each clamped to >= 0 (left edge padding of data_amass.py:30-33), root-relative.
__global__ void stream_window_kernel(const float* ring, int W, int V, const int* count, int h, int ra, int rb,
                                     int relative, float* out) {
    const int n = *count;
    const int last = n - 1;
    for (int p = threadIdx.x; p < W * V; p += blockDim.x) {
        const int k = p / V, v = p % V;
        int f = last - 2 * h + k;
        f = f < 0 ? 0 : f;
        const float* fr = ring + (size_t)(f % W) * V * 3;
        float o0 = fr[v * 3], o1 = fr[v * 3 + 1], o2 = fr[v * 3 + 2];
        if (relative) {
            o0 -= 0.5f * (fr[ra * 3] + fr[rb * 3]);
            o1 -= 0.5f * (fr[ra * 3 + 1] + fr[rb * 3 + 1]);
            o2 -= 0.5f * (fr[ra * 3 + 2] + fr[rb * 3 + 2]);
        }
        out[(size_t)p * 3] = o0;
        out[(size_t)p * 3 + 1] = o1;
        out[(size_t)p * 3 + 2] = o2;
    }
}

hipError_t launch_stream_push(float* ring, int W, int nv, int* count, const float* frame, hipStream_t st) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(stream_push_kernel, dim3(1), dim3(64), 0, st, ring, W, nv, count, frame);
    return hipGetLastError();
}

hipError_t launch_stream_window(const float* ring, int W, int V, const int* count, int h, int ra, int rb,
                                int relative, float* out, hipStream_t st) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(stream_window_kernel, dim3(1), dim3(256), 0, st, ring, W, V, count, h, ra, rb, relative, out);
    return hipGetLastError();
}

__global__ void checksum_kernel(const unsigned* __restrict__ p, size_t n, unsigned long long* out) {
    unsigned long long c = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        c += (unsigned long long)p[i] * (2 * (i & 0xffff) + 1);
    if (c) atomicAdd(out, c);
}

hipError_t launch_checksum(const void* p, size_t bytes, unsigned long long* out, hipStream_t st) {
    (void)hipGetLastError();
    hipLaunchKernelGGL(checksum_kernel, dim3(1024), dim3(256), 0, st, static_cast<const unsigned*>(p), bytes / 4, out);
    return hipGetLastError();
}

struct Map17 {
    int m[17];
};

// one thread per (frame, COCO joint): a pure gather + the axis swap, so the
// output is bit-identical to the reference's numpy (0.5 * (a + b) in fp32 is an
// exact halving of the fp32 sum, as numpy computes it on float32 arrays)
__global__ void moveai_to_coco_kernel(const float* __restrict__ j, int F, int J, Map17 mp, float* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)F * 17) return;
    const int c = (int)(i % 17);
    const long long f = i / 17;
    const float* jf = j + f * J * 3;
    float x = 0.f, y = 0.f, z = 0.f;
    if (c == 0) {
        x = 0.5f * (jf[(J - 1) * 3 + 0] + jf[(J - 2) * 3 + 0]);
        y = 0.5f * (jf[(J - 1) * 3 + 1] + jf[(J - 2) * 3 + 1]);
        z = 0.5f * (jf[(J - 1) * 3 + 2] + jf[(J - 2) * 3 + 2]);
    } else {
        const int src = c == 1 ? J - 2 : (c == 2 ? J - 1 : mp.m[c]);
        if (src >= 0) { x = jf[src * 3]; y = jf[src * 3 + 1]; z = jf[src * 3 + 2]; }
    }
    float* o = out + i * 3;
    o[0] = x;
    o[1] = z;
    o[2] = -y;
}

hipError_t launch_moveai_to_coco(const float* joints, int F, int J, const int* map17, float* out, hipStream_t st) {
    if (F <= 0) return hipSuccess;
    Map17 mp;
    for (int c = 0; c < 17; ++c) {
        if (map17[c] >= J) return hipErrorInvalidValue;
        mp.m[c] = map17[c];
    }
    const long long n = (long long)F * 17;
    (void)hipGetLastError();
    hipLaunchKernelGGL(moveai_to_coco_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, joints, F, J, mp, out);
    return hipGetLastError();
}

}  // namespace tik
