// LayerNorm2d (NAFNet_base/basicsr/models/archs/arch_util.py:264-300): per-pixel normalisation over channels,
// biased variance, y = (x - mu) / sqrt(var + eps), affine; closed-form backward (:277-289).
// NHWC: channels contiguous, G lanes per pixel, shuffle reductions.  NCHW: one thread per pixel (module API).
#include "nbp_common.h"

using namespace nbp;

namespace {

// NHWC kernels: a row (pixel) of C channels = C / E chunks of 16 bytes (E = 8 bf16 / 4 fp32 elements) spread over
// G lanes x V chunks (G a power of two, G * V >= C / E: lanes past the last chunk hold zeros and store nothing, so any
// multiple of E works); each wave handles 2 x (64 / G) rows per iteration (two independent rows per lane group for
// load-level parallelism).  The forward writes the affine output and per-row stats (mu, den = sqrt(var + eps)); the backward
// recomputes yhat = (x - mu) / den from the block input it keeps anyway, so yhat is never stored.
template <typename T>
__device__ __forceinline__ void ld_chunk(const T* p, float* f) {
  if constexpr (sizeof(T) == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  } else {
    const vec_t<T, 8> v = *reinterpret_cast<const vec_t<T, 8>*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  }
}
template <typename T>
__device__ __forceinline__ void st_chunk(T* p, const float* f) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  } else {
    vec_t<T, 8> v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (T)f[j];
    *reinterpret_cast<vec_t<T, 8>*>(p) = v;
  }
}

template <int G, int V, typename T>
__global__ __launch_bounds__(256) void ln_fwd_nhwc(const T* __restrict__ x, const float* __restrict__ w,
                                                   const float* __restrict__ b, T* __restrict__ nout,
                                                   float2* __restrict__ stats, long M, int C, float eps) {
  constexpr int E = 16 / sizeof(T), RPW = 64 / G;
  const int lane = threadIdx.x & 63, lg = lane % G, nch = C / E;
  const long wave_global = (long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const long nwaves = (long)gridDim.x * (blockDim.x / 64);
  // Loads are branch-free: lanes past the last chunk / rows past M read the last chunk / row (in bounds) and mask the
  // values to zero afterwards, so both rows' loads are in flight together (a guarded load waits inside its branch).
  bool cv[V];  // this lane's chunk j exists
  int cc[V];   // its first channel (clamped)
  float wr[V][E], br[V][E];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    cv[j] = j * G + lg < nch;
    cc[j] = (cv[j] ? j * G + lg : nch - 1) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      wr[j][e] = w[cc[j] + e];
      br[j][e] = b[cc[j] + e];
    }
  }
  for (long r0 = wave_global * 2 * RPW; r0 < M; r0 += nwaves * 2 * RPW) {
    long row[2];
    bool ok[2];
    float v[2][V][E];
    float s[2] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      row[r] = r0 + r * RPW + lane / G;
      ok[r] = row[r] < M;
      const long rl = ok[r] ? row[r] : M - 1;
#pragma unroll
      for (int j = 0; j < V; ++j) ld_chunk(x + rl * C + cc[j], v[r][j]);
    }
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int j = 0; j < V; ++j)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          v[r][j][e] = ok[r] && cv[j] ? v[r][j][e] : 0.f;
          s[r] += v[r][j][e];
        }
    s[0] = group_sum<G>(s[0]);
    s[1] = group_sum<G>(s[1]);
    float q[2] = {0.f, 0.f}, mu[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      mu[r] = s[r] / (float)C;
#pragma unroll
      for (int j = 0; j < V; ++j)
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float d = cv[j] ? v[r][j][e] - mu[r] : 0.f;
          q[r] = fmaf(d, d, q[r]);
        }
    }
    q[0] = group_sum<G>(q[0]);
    q[1] = group_sum<G>(q[1]);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!ok[r]) continue;
      const float dd = sqrtf(q[r] / (float)C + eps), inv = 1.f / dd;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if (!cv[j]) continue;
        float o[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {  // rounded to fp32 before the store conversion (no single-rounding fma_mix)
          o[e] = fmaf(wr[j][e], (v[r][j][e] - mu[r]) * inv, br[j][e]);
          asm volatile("" : "+v"(o[e]));
        }
        st_chunk(nout + row[r] * C + cc[j], o);
      }
      if (lg == 0) stats[row[r]] = make_float2(mu[r], dd);
    }
  }
}

// dx = (g - yhat * mean(g * yhat) - mean(g)) / den + dres,  g = dn * w,  yhat = (x - mu) / den;
// per-block partials of sum(dn * yhat) and sum(dn) into slab_w / slab_b ([grid][C], fixed-order fold)
template <int G, int V, typename T>
__global__ __launch_bounds__(256) void ln_bwd_nhwc(const T* __restrict__ dn, const T* __restrict__ x,
                                                   const float2* __restrict__ stats, const float* __restrict__ w,
                                                   const T* __restrict__ dres, T* __restrict__ dx,
                                                   float* __restrict__ slab_w, float* __restrict__ slab_b, long M,
                                                   int C) {
  constexpr int E = 16 / sizeof(T), RPW = 64 / G, CMAX = G * V * E;
  constexpr bool PRE = V <= 2;  // dres loaded with dn / x (its chunks held raw; wider rows load it at the store)
  __shared__ float red[4][2][CMAX];
  const int lane = threadIdx.x & 63, lg = lane % G, wv = threadIdx.x >> 6, nch = C / E;
  const long wave_global = (long)blockIdx.x * (blockDim.x / 64) + wv;
  const long nwaves = (long)gridDim.x * (blockDim.x / 64);
  const T* rp = dres ? dres : dn;  // branch-free residual loads (ignored without dres)
  bool cv[V];  // branch-free loads as in ln_fwd_nhwc: clamped chunk / row, values masked
  int cc[V];
  float aw[V][E], ab[V][E];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    cv[j] = j * G + lg < nch;
    cc[j] = (cv[j] ? j * G + lg : nch - 1) * E;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      aw[j][e] = ab[j][e] = 0.f;
    }
  }
  for (long r0 = wave_global * 2 * RPW; r0 < M; r0 += nwaves * 2 * RPW) {
    long row[2], rl[2];
    bool ok[2];
    float d[2][V][E], yh[2][V][E], wr[V][E];
    vec_t<T, E> rres[2][PRE ? V : 1];
#pragma unroll
    for (int j = 0; j < V; ++j) {  // weights reloaded per row pair (cache hits), issued with the rows: a copy hoisted
      int ci = cc[j];              // out of the loop waits for them before the first row loads
      asm volatile("" : "+v"(ci));
#pragma unroll
      for (int e = 0; e < E; ++e) wr[j][e] = w[ci + e];  // (unmasked: g is masked below)
    }
    float2 st[2];
    float sg[2] = {0.f, 0.f}, sgy[2] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      row[r] = r0 + r * RPW + lane / G;
      ok[r] = row[r] < M;
      rl[r] = ok[r] ? row[r] : M - 1;
      st[r] = stats[rl[r]];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        ld_chunk(dn + rl[r] * C + cc[j], d[r][j]);
        ld_chunk(x + rl[r] * C + cc[j], yh[r][j]);
        if constexpr (PRE) rres[r][j] = *reinterpret_cast<const vec_t<T, E>*>(rp + rl[r] * C + cc[j]);
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!ok[r]) st[r] = make_float2(0.f, 1.f);
#pragma unroll
      for (int j = 0; j < V; ++j)
#pragma unroll
        for (int e = 0; e < E; ++e) d[r][j][e] = ok[r] && cv[j] ? d[r][j][e] : 0.f;
    }
    const float rinv[2] = {1.f / st[0].y, 1.f / st[1].y};
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int j = 0; j < V; ++j) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float y = ok[r] && cv[j] ? (yh[r][j][e] - st[r].x) * rinv[r] : 0.f;
          yh[r][j][e] = y;
          const float wm = cv[j] ? wr[j][e] : 0.f;
          const float g = d[r][j][e] * wm;
          sg[r] = fmaf(d[r][j][e], wm, sg[r]);  // (the contraction of sg += g the compiler chose, spelt out)
          sgy[r] = fmaf(g, y, sgy[r]);
          aw[j][e] = fmaf(d[r][j][e], y, aw[j][e]);
          ab[j][e] += d[r][j][e];
        }
      }
    sg[0] = group_sum<G>(sg[0]);
    sg[1] = group_sum<G>(sg[1]);
    sgy[0] = group_sum<G>(sgy[0]);
    sgy[1] = group_sum<G>(sgy[1]);
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      if (!ok[r]) continue;
      const float mg = sg[r] / (float)C, mgy = sgy[r] / (float)C, inv = rinv[r];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        if (!cv[j]) continue;
        float o[E], rr[E];
        if constexpr (PRE) {
#pragma unroll
          for (int e = 0; e < E; ++e) rr[e] = (float)rres[r][j][e];
        } else {
          ld_chunk(rp + row[r] * C + cc[j], rr);
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {  // the contraction the compiler chose for (g - yhat * mgy - mg) * inv + dres, spelt out
          const float t = fmaf(-yh[r][j][e], mgy, d[r][j][e] * wr[j][e]) - mg;
          o[e] = dres ? fmaf(inv, t, rr[e]) : t * inv;
        }
        st_chunk(dx + row[r] * C + cc[j], o);
      }
    }
  }
  // fold the partials over lanes sharing lg, then over the block's waves (fixed order)
#pragma unroll
  for (int j = 0; j < V; ++j)
#pragma unroll
    for (int e = 0; e < E; ++e) {
#pragma unroll
      for (int o = G; o < 64; o <<= 1) {
        aw[j][e] += __shfl_xor(aw[j][e], o, 64);
        ab[j][e] += __shfl_xor(ab[j][e], o, 64);
      }
      if (lane < G && cv[j]) {
        red[wv][0][(j * G + lg) * E + e] = aw[j][e];
        red[wv][1][(j * G + lg) * E + e] = ab[j][e];
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

int ln_lanes(int chunks) {  // G: the power of two >= the chunk count, at most 64
  int G = 1;
  while (G < chunks && G < 64) G <<= 1;
  return G;
}

int ln_grid(long M, int C, int dtype) {
  const int G = ln_lanes(C / (dtype != 0 ? 8 : 4));
  const long rows_per_block = 4L * 2 * (64 / G);
  long g = (M + rows_per_block - 1) / rows_per_block;
  if (g > 1024) g = 1024;
  return (int)(g < 1 ? 1 : g);
}

// (G, V) from the chunk count n = C / E: G = the power of two >= n (at most 64), V = ceil(n / 64) in {1, 2, 4}
#define NBP_LN_DISPATCH(KERNEL, ...)                                                          \
  switch (C / E <= 64 ? ln_lanes(C / E) : (C / E <= 128 ? 128 : 256)) {                       \
    case 1: KERNEL<1, 1, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                           \
    case 2: KERNEL<2, 1, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                           \
    case 4: KERNEL<4, 1, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                           \
    case 8: KERNEL<8, 1, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                           \
    case 16: KERNEL<16, 1, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                         \
    case 32: KERNEL<32, 1, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                         \
    case 64: KERNEL<64, 1, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                         \
    case 128: KERNEL<64, 2, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                        \
    default: KERNEL<64, 4, T><<<g, 256, 0, st>>>(__VA_ARGS__); break;                         \
  }

}  // namespace

extern "C" {

int nbp_ln_nhwc_grid(long M, int C, int dtype) { return ln_grid(M, C, dtype); }

int nbp_ln_fwd_nhwc(const void* x, const float* w, const float* b, void* nout, float* stats, long M, int C, float eps,
                    int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && w && b && nout && stats && M > 0, "nbp_ln_fwd_nhwc: bad args");
  const int E = dtype != 0 ? 8 : 4;
  NBP_REQUIRE(C >= E && C / E <= 256 && C % E == 0, "nbp_ln_fwd_nhwc: C must be a multiple of %d in [%d, %d]", E,
              E, 256 * E);
  const int g = ln_grid(M, C, dtype);
  hipStream_t st = S(s);
  NBP_DISPATCH_T(dtype, {
    NBP_LN_DISPATCH(ln_fwd_nhwc, (const T*)x, w, b, (T*)nout, reinterpret_cast<float2*>(stats), M, C, eps);
  });
  return check_launch("ln_fwd_nhwc");
}

// slab_w / slab_b: [nbp_ln_nhwc_grid(M, C, dtype)][C] floats each; reduced by the caller (nbp_reduce_slab)
int nbp_ln_bwd_nhwc(const void* dn, const void* x, const float* stats, const float* w, const void* dres, void* dx,
                    float* slab_w, float* slab_b, long M, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dn && x && stats && w && dx && slab_w && slab_b && M > 0, "nbp_ln_bwd_nhwc: bad args");
  const int E = dtype != 0 ? 8 : 4;
  NBP_REQUIRE(C >= E && C / E <= 256 && C % E == 0, "nbp_ln_bwd_nhwc: C must be a multiple of %d in [%d, %d]", E,
              E, 256 * E);
  const int g = ln_grid(M, C, dtype);
  hipStream_t st = S(s);
  NBP_DISPATCH_T(dtype, {
    NBP_LN_DISPATCH(ln_bwd_nhwc, (const T*)dn, (const T*)x, reinterpret_cast<const float2*>(stats), w, (const T*)dres,
                    (T*)dx, slab_w, slab_b, M, C);
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
