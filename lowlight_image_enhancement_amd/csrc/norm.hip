// LayerNorm2d (NAFNet_base/basicsr/models/archs/arch_util.py:264-300): per-pixel normalisation over channels,
// biased variance, y = (x - mu) / sqrt(var + eps), affine; closed-form backward (:277-289).
// NHWC: channels contiguous, G lanes per pixel, shuffle reductions.  NCHW: one thread per pixel (module API).
#include "nbp_common.h"

using namespace nbp;

namespace {

constexpr int kMaxV = 4;  // C <= 4 * 4 * 64 = 1024

template <int G, typename T>
__global__ __launch_bounds__(256) void ln_fwd_nhwc(const T* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ b, T* __restrict__ yhat,
                                                   T* __restrict__ nout, float* __restrict__ den, long M, int C,
                                                   float eps) {
  const int lane = threadIdx.x & 63, lg = lane % G;
  constexpr int RPW = 64 / G;
  const int V = C / (4 * G);
  const long wave_global = (long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const long nwaves = (long)gridDim.x * (blockDim.x / 64);
  for (long r0 = wave_global * RPW; r0 < M; r0 += nwaves * RPW) {
    const long row = r0 + lane / G;
    const bool ok = row < M;
    float4 v[kMaxV];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxV; ++j) {
      if (j < V) {
        v[j] = ok ? ldq(x + row * C + (j * G + lg) * 4) : f4(0.f);
        s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
      }
    }
    s = group_sum<G>(s);
    const float mu = s / (float)C;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxV; ++j) {
      if (j < V) {
        const float4 d = v[j] - f4(mu);
        q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
      }
    }
    q = group_sum<G>(q);
    const float var = q / (float)C;
    const float dd = sqrtf(var + eps);
    if (!ok) continue;
#pragma unroll
    for (int j = 0; j < kMaxV; ++j) {
      if (j < V) {
        const int c = (j * G + lg) * 4;
        const float4 d = v[j] - f4(mu);
        const float4 yh = make_float4(d.x / dd, d.y / dd, d.z / dd, d.w / dd);
        if (yhat) stq(yhat + row * C + c, yh);
        stq(nout + row * C + c, fma4(ld4(w + c), yh, ld4(b + c)));
      }
    }
    if (lg == 0) den[row] = dd;
  }
}

// dx = (g - yhat * mean(g*yhat) - mean(g)) / den + dres,  g = dn * w;  per-block partials of sum(dn*yhat), sum(dn)
template <int G, typename T>
__global__ __launch_bounds__(256) void ln_bwd_nhwc(const T* __restrict__ dn, const T* __restrict__ yhat,
                                                   const float* __restrict__ den, const float* __restrict__ w,
                                                   const T* __restrict__ dres, T* __restrict__ dx,
                                                   float* __restrict__ slab_w, float* __restrict__ slab_b, long M,
                                                   int C) {
  __shared__ float red[4][2][1024];
  const int lane = threadIdx.x & 63, lg = lane % G, wv = threadIdx.x >> 6;
  constexpr int RPW = 64 / G;
  const int V = C / (4 * G);
  const long wave_global = (long)blockIdx.x * (blockDim.x / 64) + wv;
  const long nwaves = (long)gridDim.x * (blockDim.x / 64);
  float4 aw[kMaxV], ab[kMaxV];
#pragma unroll
  for (int j = 0; j < kMaxV; ++j) aw[j] = ab[j] = f4(0.f);
  for (long r0 = wave_global * RPW; r0 < M; r0 += nwaves * RPW) {
    const long row = r0 + lane / G;
    const bool ok = row < M;
    float4 g[kMaxV], yh[kMaxV];
    float sg = 0.f, sgy = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxV; ++j) {
      if (j < V) {
        const int c = (j * G + lg) * 4;
        const float4 d = ok ? ldq(dn + row * C + c) : f4(0.f);
        yh[j] = ok ? ldq(yhat + row * C + c) : f4(0.f);
        g[j] = d * ld4(w + c);
        aw[j] = fma4(d, yh[j], aw[j]);
        ab[j] += d;
        sg += (g[j].x + g[j].y) + (g[j].z + g[j].w);
        const float4 gy = g[j] * yh[j];
        sgy += (gy.x + gy.y) + (gy.z + gy.w);
      }
    }
    sg = group_sum<G>(sg);
    sgy = group_sum<G>(sgy);
    if (!ok) continue;
    const float mg = sg / (float)C, mgy = sgy / (float)C;
    const float inv = 1.f / den[row];
#pragma unroll
    for (int j = 0; j < kMaxV; ++j) {
      if (j < V) {
        const int c = (j * G + lg) * 4;
        float4 o = (g[j] - yh[j] * f4(mgy) - f4(mg)) * f4(inv);
        if (dres) o += ldq(dres + row * C + c);
        stq(dx + row * C + c, o);
      }
    }
  }
  // reduce partials over lanes sharing lg, then over the block's waves
#pragma unroll
  for (int j = 0; j < kMaxV; ++j) {
    if (j < V) {
#pragma unroll
      for (int o = G; o < 64; o <<= 1) {
        aw[j].x += __shfl_xor(aw[j].x, o, 64); aw[j].y += __shfl_xor(aw[j].y, o, 64);
        aw[j].z += __shfl_xor(aw[j].z, o, 64); aw[j].w += __shfl_xor(aw[j].w, o, 64);
        ab[j].x += __shfl_xor(ab[j].x, o, 64); ab[j].y += __shfl_xor(ab[j].y, o, 64);
        ab[j].z += __shfl_xor(ab[j].z, o, 64); ab[j].w += __shfl_xor(ab[j].w, o, 64);
      }
      if (lane < G) {
        const int c = (j * G + lg) * 4;
        st4(&red[wv][0][c], aw[j]);
        st4(&red[wv][1][c], ab[j]);
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float sw = 0.f, sb = 0.f;
    for (int k = 0; k < (int)(blockDim.x / 64); ++k) {
      sw += red[k][0][c];
      sb += red[k][1][c];
    }
    slab_w[(long)blockIdx.x * C + c] = sw;
    slab_b[(long)blockIdx.x * C + c] = sb;
  }
}

// NCHW (standalone LayerNorm2d module): one thread per pixel, loops over channels with stride HW
__global__ void ln_fwd_nchw(const float* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                            float* __restrict__ y, float* __restrict__ yhat, float* __restrict__ den, int N, int C,
                            long HW, float eps) {
  const long total = (long)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW, p = i % HW;
    const float* xp = x + n * C * HW + p;
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += xp[c * HW];
    const float mu = s / (float)C;
    float q = 0.f;
    for (int c = 0; c < C; ++c) {
      const float d = xp[c * HW] - mu;
      q += d * d;
    }
    const float dd = sqrtf(q / (float)C + eps);
    for (int c = 0; c < C; ++c) {
      const float yh = (xp[c * HW] - mu) / dd;
      yhat[n * C * HW + c * HW + p] = yh;
      y[n * C * HW + c * HW + p] = fmaf(w[c], yh, b[c]);
    }
    den[i] = dd;
  }
}

__global__ void ln_bwd_nchw(const float* __restrict__ dy, const float* __restrict__ yhat, const float* __restrict__ den,
                            const float* __restrict__ w, float* __restrict__ dx, int N, int C, long HW) {
  const long total = (long)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW, p = i % HW;
    const long base = n * C * HW + p;
    float sg = 0.f, sgy = 0.f;
    for (int c = 0; c < C; ++c) {
      const float g = dy[base + c * HW] * w[c];
      sg += g;
      sgy += g * yhat[base + c * HW];
    }
    const float mg = sg / (float)C, mgy = sgy / (float)C, inv = 1.f / den[i];
    for (int c = 0; c < C; ++c) {
      const float g = dy[base + c * HW] * w[c];
      dx[base + c * HW] = (g - yhat[base + c * HW] * mgy - mg) * inv;
    }
  }
}

// per-channel partial sums over NCHW: slab_w[blk][c] = sum dy*yhat, slab_b[blk][c] = sum dy  (grid.y = channel)
__global__ void ln_wb_nchw(const float* __restrict__ dy, const float* __restrict__ yhat, int N, int C, long HW,
                           float* __restrict__ slab_w, float* __restrict__ slab_b) {
  __shared__ double red[16];
  const int c = blockIdx.y;
  double sw = 0.0, sb = 0.0;
  const long total = (long)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / HW, p = i % HW;
    const long o = n * C * HW + (long)c * HW + p;
    sw += (double)dy[o] * yhat[o];
    sb += dy[o];
  }
  sw = block_sum_d(sw, red);
  sb = block_sum_d(sb, red);
  if (threadIdx.x == 0) {
    slab_w[(long)blockIdx.x * C + c] = (float)sw;
    slab_b[(long)blockIdx.x * C + c] = (float)sb;
  }
}

template <int G>
int ln_grid(long M) {
  const long rows_per_block = 4L * (64 / G);
  long g = (M + rows_per_block - 1) / rows_per_block;
  if (g > 1024) g = 1024;
  return (int)(g < 1 ? 1 : g);
}

int pick_G(int C) {
  const int q = C / 4;
  return q >= 64 ? 64 : q;
}

}  // namespace

extern "C" {

int nbp_ln_nhwc_grid(long M, int C) {
  switch (pick_G(C)) {
    case 64: return ln_grid<64>(M);
    case 32: return ln_grid<32>(M);
    case 16: return ln_grid<16>(M);
    case 8: return ln_grid<8>(M);
    case 4: return ln_grid<4>(M);
    default: return ln_grid<2>(M);
  }
}

int nbp_ln_fwd_nhwc(const void* x, const float* w, const float* b, void* yhat, void* nout, float* den, long M, int C,
                    float eps, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && w && b && nout && den && M > 0, "nbp_ln_fwd_nhwc: bad args");
  NBP_REQUIRE(C >= 8 && C <= 1024 && (C & (C - 1)) == 0, "nbp_ln_fwd_nhwc: C must be a power of two in [8,1024]");
  const int g = nbp_ln_nhwc_grid(M, C);
  hipStream_t st = S(s);
  NBP_DISPATCH_T(dtype, {
    const T* xx = (const T*)x;
    T* yy = (T*)yhat;
    T* nn = (T*)nout;
    switch (pick_G(C)) {
      case 64: ln_fwd_nhwc<64, T><<<g, 256, 0, st>>>(xx, w, b, yy, nn, den, M, C, eps); break;
      case 32: ln_fwd_nhwc<32, T><<<g, 256, 0, st>>>(xx, w, b, yy, nn, den, M, C, eps); break;
      case 16: ln_fwd_nhwc<16, T><<<g, 256, 0, st>>>(xx, w, b, yy, nn, den, M, C, eps); break;
      case 8: ln_fwd_nhwc<8, T><<<g, 256, 0, st>>>(xx, w, b, yy, nn, den, M, C, eps); break;
      case 4: ln_fwd_nhwc<4, T><<<g, 256, 0, st>>>(xx, w, b, yy, nn, den, M, C, eps); break;
      default: ln_fwd_nhwc<2, T><<<g, 256, 0, st>>>(xx, w, b, yy, nn, den, M, C, eps); break;
    }
  });
  return check_launch("ln_fwd_nhwc");
}

// slab_w / slab_b: [grid][C] floats each (grid = nbp_ln_nhwc_grid(M, C)); reduced by the caller (nbp_reduce_slab)
int nbp_ln_bwd_nhwc(const void* dn, const void* yhat, const float* den, const float* w, const void* dres, void* dx,
                    float* slab_w, float* slab_b, long M, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dn && yhat && den && w && dx && slab_w && slab_b && M > 0, "nbp_ln_bwd_nhwc: bad args");
  NBP_REQUIRE(C >= 8 && C <= 1024 && (C & (C - 1)) == 0, "nbp_ln_bwd_nhwc: C must be a power of two in [8,1024]");
  const int g = nbp_ln_nhwc_grid(M, C);
  hipStream_t st = S(s);
  NBP_DISPATCH_T(dtype, {
    const T* a = (const T*)dn;
    const T* yh = (const T*)yhat;
    const T* r = (const T*)dres;
    T* o = (T*)dx;
    switch (pick_G(C)) {
      case 64: ln_bwd_nhwc<64, T><<<g, 256, 0, st>>>(a, yh, den, w, r, o, slab_w, slab_b, M, C); break;
      case 32: ln_bwd_nhwc<32, T><<<g, 256, 0, st>>>(a, yh, den, w, r, o, slab_w, slab_b, M, C); break;
      case 16: ln_bwd_nhwc<16, T><<<g, 256, 0, st>>>(a, yh, den, w, r, o, slab_w, slab_b, M, C); break;
      case 8: ln_bwd_nhwc<8, T><<<g, 256, 0, st>>>(a, yh, den, w, r, o, slab_w, slab_b, M, C); break;
      case 4: ln_bwd_nhwc<4, T><<<g, 256, 0, st>>>(a, yh, den, w, r, o, slab_w, slab_b, M, C); break;
      default: ln_bwd_nhwc<2, T><<<g, 256, 0, st>>>(a, yh, den, w, r, o, slab_w, slab_b, M, C); break;
    }
  });
  return check_launch("ln_bwd_nhwc");
}

int nbp_ln_fwd_nchw(const float* x, const float* w, const float* b, float* y, float* yhat, float* den, int N, int C,
                    long HW, float eps, nbp_stream_t s) {
  NBP_REQUIRE(x && w && b && y && yhat && den && N > 0 && C > 0 && HW > 0, "nbp_ln_fwd_nchw: bad args");
  long g = ((long)N * HW + 255) / 256;
  ln_fwd_nchw<<<(int)(g > 4096 ? 4096 : g), 256, 0, S(s)>>>(x, w, b, y, yhat, den, N, C, HW, eps);
  return check_launch("ln_fwd_nchw");
}

int nbp_ln_bwd_nchw_workspace_floats(int N, int C, long HW) { return 2 * 64 * C; }

int nbp_ln_bwd_nchw(const float* dy, const float* yhat, const float* den, const float* w, float* dx, float* dw,
                    float* db, float* ws, int N, int C, long HW, nbp_stream_t s) {
  NBP_REQUIRE(dy && yhat && den && w && dx && dw && db && ws && N > 0 && C > 0 && HW > 0, "nbp_ln_bwd_nchw: bad args");
  hipStream_t st = S(s);
  long g = ((long)N * HW + 255) / 256;
  ln_bwd_nchw<<<(int)(g > 4096 ? 4096 : g), 256, 0, st>>>(dy, yhat, den, w, dx, N, C, HW);
  ln_wb_nchw<<<dim3(64, C), 256, 0, st>>>(dy, yhat, N, C, HW, ws, ws + 64 * C);
  int rc = nbp_reduce_slab(ws, 64, C, dw, s);
  if (rc) return rc;
  rc = nbp_reduce_slab(ws + 64 * C, 64, C, db, s);
  if (rc) return rc;
  return check_launch("ln_bwd_nchw");
}

}  // extern "C"
