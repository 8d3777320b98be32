// Elementwise and per-channel reduction kernels on NHWC activations:
//   SimpleGate fwd/bwd for the FFN half of NAFBlock (NAFNet_arch.py:22-25,74-76),
//   the layer-scale residual gradients dbeta/dgamma (NAFNet_arch.py:56-57,72,80) and NCHW<->NHWC transposes.
#include "nbp_common.h"

using namespace nbp;

namespace {

// layout 0: t = [first half | second half] (g = t[:C] * t[C:]); layout 1: channel pairs interleaved
// (g[c] = t[2c] * t[2c+1]) — the order of the fused-epilogue path (conv4's rows stored interleaved)
template <typename T>
__global__ void sg_fwd(const T* __restrict__ t, T* __restrict__ g, long M, int C, int layout) {
  const int Q = C / 4;
  const long total = M * Q;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long m = e / Q;
    const int q = e % Q;
    if (layout == 0) {
      stq(g + m * C + q * 4, ldq(t + m * 2 * C + q * 4) * ldq(t + m * 2 * C + C + q * 4));
    } else {
      const float4 a = ldq(t + m * 2 * C + q * 8), b = ldq(t + m * 2 * C + q * 8 + 4);
      stq(g + m * C + q * 4, make_float4(a.x * a.y, a.z * a.w, b.x * b.y, b.z * b.w));
    }
  }
}

template <typename T>
__global__ void sg_bwd(const T* __restrict__ dg, const T* __restrict__ t, T* __restrict__ dt, long M, int C,
                       int layout) {
  const int Q = C / 4;
  const long total = M * Q;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long m = e / Q;
    const int q = e % Q;
    const float4 d = ldq(dg + m * C + q * 4);
    if (layout == 0) {
      const float4 a = ldq(t + m * 2 * C + q * 4), b = ldq(t + m * 2 * C + C + q * 4);
      stq(dt + m * 2 * C + q * 4, d * b);
      stq(dt + m * 2 * C + C + q * 4, d * a);
    } else {
      const float4 a = ldq(t + m * 2 * C + q * 8), b = ldq(t + m * 2 * C + q * 8 + 4);
      stq(dt + m * 2 * C + q * 8, make_float4(d.x * a.y, d.x * a.x, d.y * a.w, d.y * a.z));
      stq(dt + m * 2 * C + q * 8 + 4, make_float4(d.z * b.y, d.z * b.x, d.w * b.w, d.w * b.z));
    }
  }
}

// ds[m][c] = d[m][c] * scale[c] ; slab[blk][c] = sum_m d[m][c] * t[m][c]
template <typename T>
__global__ void scale_dot(const T* __restrict__ d, const T* __restrict__ t, const float* __restrict__ scale,
                          T* __restrict__ ds, float* __restrict__ slab, long M, int C) {
  extern __shared__ float red[];
  const int Q = C / 4;
  const int tid = threadIdx.x, q = tid % Q, rl = tid / Q, RPS = blockDim.x / Q;
  float4 acc = f4(0.f);
  const float4 sc = ld4(scale + q * 4);
  if (rl < RPS) {
    for (long m = (long)blockIdx.x * RPS + rl; m < M; m += (long)gridDim.x * RPS) {
      const float4 dv = ldq(d + m * C + q * 4);
      acc = fma4(dv, ldq(t + m * C + q * 4), acc);
      stq(ds + m * C + q * 4, dv * sc);
    }
  }
  st4(red + tid * 4, acc);
  __syncthreads();
  if (rl == 0) {
    float4 s = f4(0.f);
    for (int k = 0; k < RPS; ++k) s += ld4(red + (k * Q + q) * 4);
    st4(slab + (long)blockIdx.x * C + q * 4, s);
  }
}

// NCHW [N][C][HW] -> NHWC [N][HW][C] via a 32x32 LDS tile
__global__ void nchw_to_nhwc(const float* __restrict__ x, float* __restrict__ y, int C, long HW) {
  __shared__ float tile[32][33];
  const int n = blockIdx.z;
  const long p0 = (long)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 rows per pass
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r;
    const long p = p0 + tx;
    tile[r][tx] = (c < C && p < HW) ? x[((long)n * C + c) * HW + p] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const long p = p0 + r;
    const int c = c0 + tx;
    if (c < C && p < HW) y[((long)n * HW + p) * C + c] = tile[tx][r];
  }
}

__global__ void nhwc_to_nchw(const float* __restrict__ x, float* __restrict__ y, int C, long HW) {
  __shared__ float tile[32][33];
  const int n = blockIdx.z;
  const long p0 = (long)blockIdx.x * 32;
  const int c0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const long p = p0 + r;
    const int c = c0 + tx;
    tile[r][tx] = (c < C && p < HW) ? x[((long)n * HW + p) * C + c] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int c = c0 + r;
    const long p = p0 + tx;
    if (c < C && p < HW) y[((long)n * C + c) * HW + p] = tile[tx][r];
  }
}

template <typename T>
__global__ void add_kernel(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = (T)((float)a[i] + (float)b[i]);
}

inline int g_elem(long total) {
  long g = (total + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

int nbp_sg_fwd(const void* t, void* g, long M, int C, int layout, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(t && g && M > 0 && C % 4 == 0 && (layout == 0 || layout == 1), "nbp_sg_fwd: bad args");
  NBP_DISPATCH_T(dtype, sg_fwd<T><<<g_elem(M * (C / 4)), 256, 0, S(s)>>>((const T*)t, (T*)g, M, C, layout));
  return check_launch("sg_fwd");
}

int nbp_sg_bwd(const void* dg, const void* t, void* dt, long M, int C, int layout, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dg && t && dt && M > 0 && C % 4 == 0 && (layout == 0 || layout == 1), "nbp_sg_bwd: bad args");
  NBP_DISPATCH_T(dtype, sg_bwd<T><<<g_elem(M * (C / 4)), 256, 0, S(s)>>>((const T*)dg, (const T*)t, (T*)dt, M, C,
                                                                         layout));
  return check_launch("sg_bwd");
}

int nbp_scale_dot_grid(long M, int C) {
  const int Q = C / 4;
  const int rps = Q >= 256 ? 1 : 256 / Q;
  long g = (M + rps - 1) / rps;
  return (int)(g > 1024 ? 1024 : (g < 1 ? 1 : g));
}

// slab: [nbp_scale_dot_grid(M, C)][C]
int nbp_scale_dot(const void* d, const void* t, const float* scale, void* ds, float* slab, long M, int C, int dtype,
                  nbp_stream_t s) {
  NBP_REQUIRE(d && t && scale && ds && slab && M > 0 && C % 4 == 0 && C / 4 <= 1024, "nbp_scale_dot: bad args");
  const int Q = C / 4, blk = Q >= 256 ? Q : 256;
  NBP_DISPATCH_T(dtype, scale_dot<T><<<nbp_scale_dot_grid(M, C), blk, blk * 4 * sizeof(float), S(s)>>>(
                            (const T*)d, (const T*)t, scale, (T*)ds, slab, M, C));
  return check_launch("scale_dot");
}

int nbp_nchw_to_nhwc(const float* x, float* y, int N, int C, long HW, nbp_stream_t s) {
  NBP_REQUIRE(x && y && N > 0 && C > 0 && HW > 0, "nbp_nchw_to_nhwc: bad args");
  nchw_to_nhwc<<<dim3(cdiv(HW, 32), cdiv(C, 32), N), 256, 0, S(s)>>>(x, y, C, HW);
  return check_launch("nchw_to_nhwc");
}

int nbp_nhwc_to_nchw(const float* x, float* y, int N, int C, long HW, nbp_stream_t s) {
  NBP_REQUIRE(x && y && N > 0 && C > 0 && HW > 0, "nbp_nhwc_to_nchw: bad args");
  nhwc_to_nchw<<<dim3(cdiv(HW, 32), cdiv(C, 32), N), 256, 0, S(s)>>>(x, y, C, HW);
  return check_launch("nhwc_to_nchw");
}

int nbp_add(const void* a, const void* b, void* y, long n, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(a && b && y && n > 0, "nbp_add: bad args");
  NBP_DISPATCH_T(dtype, add_kernel<T><<<g_elem(n), 256, 0, S(s)>>>((const T*)a, (const T*)b, (T*)y, n));
  return check_launch("add");
}

}  // extern "C"
