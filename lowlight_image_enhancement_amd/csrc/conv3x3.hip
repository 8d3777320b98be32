// NAFNet image-boundary convolutions (NAFNet_arch.py:88-91,134-136,152-162):
//   intro : 3x3 pad 1, img_channel -> width, on the input zero-padded to a multiple of 2^len(enc) (check_image_size);
//           reads the NCHW image, writes NHWC features on the padded grid.
//   ending: 3x3 pad 1, width -> img_channel on the padded grid, + global residual, cropped to the input size;
//           reads NHWC features, writes the NCHW image.
#include "nbp_common.h"

using namespace nbp;

namespace {

constexpr int kMaxCin = 4;  // img_channel <= 4 (kernels are instantiated for 1..4)

struct Img {
  int B, Cimg, H0, W0;  // image (unpadded)
  int Hp, Wp;           // padded feature grid
  int Cf;               // feature channels (width)
};

// ------------------------------------------------------------------ intro forward
template <int CI, typename T>
__global__ __launch_bounds__(256) void intro_fwd(const float* __restrict__ img, const float* __restrict__ w,
                                                 const float* __restrict__ bias, T* __restrict__ out, Img g) {
  extern __shared__ float wl[];  // [Cf][CI*9]
  constexpr int K = CI * 9;
  for (int i = threadIdx.x; i < g.Cf * K; i += blockDim.x) wl[i] = w[i];
  __syncthreads();
  const long total = (long)g.B * g.Hp * g.Wp;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const int x = p % g.Wp, y = (p / g.Wp) % g.Hp, b = p / ((long)g.Wp * g.Hp);
    float in[K];
#pragma unroll
    for (int c = 0; c < CI; ++c)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        in[c * 9 + t] = (yy >= 0 && yy < g.H0 && xx >= 0 && xx < g.W0)
                            ? img[(((long)b * CI + c) * g.H0 + yy) * g.W0 + xx] : 0.f;
      }
    T* op = out + p * g.Cf;
    for (int o = 0; o < g.Cf; o += 4) {
      float r[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float acc = bias[o + j];
        const float* wr = wl + (o + j) * K;
#pragma unroll
        for (int k = 0; k < K; ++k) acc = fmaf(wr[k], in[k], acc);
        r[j] = acc;
      }
      stq(op + o, make_float4(r[0], r[1], r[2], r[3]));
    }
  }
}

// intro weight gradient: slab_w[blk][Cf][CI*9], slab_b[blk][Cf]
template <int CI, typename T>
__global__ __launch_bounds__(256) void intro_bwd_w(const float* __restrict__ img, const T* __restrict__ dout, float* __restrict__ slab_w,
                            float* __restrict__ slab_b, Img g, long px_per_blk) {
  extern __shared__ float red[];  // [blockDim][4]
  constexpr int K = CI * 9;
  const int Q = g.Cf / 4;
  const int tid = threadIdx.x, q = tid % Q, pl = tid / Q, PPI = blockDim.x / Q;
  float4 acc[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) acc[k] = f4(0.f);
  const long total = (long)g.B * g.Hp * g.Wp;
  const long p0 = blockIdx.x * px_per_blk, p1 = min(total, p0 + px_per_blk);
  if (pl < PPI) {
    for (long p = p0 + pl; p < p1; p += PPI) {
      const int x = p % g.Wp, y = (p / g.Wp) % g.Hp, b = p / ((long)g.Wp * g.Hp);
      const float4 d = ldq(dout + p * g.Cf + q * 4);
      acc[K] += d;
#pragma unroll
      for (int c = 0; c < CI; ++c)
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
          const float v = (yy >= 0 && yy < g.H0 && xx >= 0 && xx < g.W0)
                              ? img[(((long)b * CI + c) * g.H0 + yy) * g.W0 + xx] : 0.f;
          acc[c * 9 + t] = fma4(d, f4(v), acc[c * 9 + t]);
        }
    }
  }
  float* dw = slab_w + (long)blockIdx.x * g.Cf * K;
  float* db = slab_b + (long)blockIdx.x * g.Cf;
#pragma unroll
  for (int kk = 0; kk <= K; ++kk) {
    st4(red + tid * 4, acc[kk]);
    __syncthreads();
    if (pl == 0) {
      float4 s4 = f4(0.f);
      for (int i = 0; i < PPI; ++i) s4 += ld4(red + (i * Q + q) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (kk < K) dw[(long)(q * 4 + j) * K + kk] = get(s4, j);
        else db[q * 4 + j] = get(s4, j);
      }
    }
    __syncthreads();
  }
}

// intro input gradient (only when the image requires grad): d img = conv^T over the padded grid, restricted to H0 x W0
template <typename T>
__global__ void intro_bwd_x(const T* __restrict__ dout, const float* __restrict__ w, float* __restrict__ dimg, Img g) {
  const long total = (long)g.B * g.Cimg * g.H0 * g.W0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = i % g.W0, y = (i / g.W0) % g.H0;
    const int c = (i / ((long)g.W0 * g.H0)) % g.Cimg;
    const int b = i / ((long)g.W0 * g.H0 * g.Cimg);
    float a = 0.f;
    for (int t = 0; t < 9; ++t) {
      const int yo = y - (t / 3 - 1), xo = x - (t % 3 - 1);
      if (yo < 0 || yo >= g.Hp || xo < 0 || xo >= g.Wp) continue;
      const T* dp = dout + (((long)b * g.Hp + yo) * g.Wp + xo) * g.Cf;
      for (int o = 0; o < g.Cf; ++o) a = fmaf(w[((long)o * g.Cimg + c) * 9 + t], (float)dp[o], a);
    }
    dimg[i] = a;
  }
}

// ------------------------------------------------------------------ ending forward
// wl layout: [t][Cf][4] with o < Cimg (<= 4) in the last dimension
template <typename T>
__global__ void ending_fwd(const T* __restrict__ feat, const float* __restrict__ w, const float* __restrict__ bias,
                           const float* __restrict__ img, float* __restrict__ out, Img g) {
  extern __shared__ float wl[];
  for (int i = threadIdx.x; i < 9 * g.Cf * 4; i += blockDim.x) {
    const int o = i & 3, c = (i >> 2) % g.Cf, t = (i >> 2) / g.Cf;
    wl[i] = o < g.Cimg ? w[((long)o * g.Cf + c) * 9 + t] : 0.f;
  }
  __syncthreads();
  const long total = (long)g.B * g.H0 * g.W0;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const int x = p % g.W0, y = (p / g.W0) % g.H0, b = p / ((long)g.W0 * g.H0);
    float4 acc = f4(0.f);
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if (yy < 0 || yy >= g.Hp || xx < 0 || xx >= g.Wp) continue;
      const T* fp = feat + (((long)b * g.Hp + yy) * g.Wp + xx) * g.Cf;
      const float* wt = wl + t * g.Cf * 4;
      for (int c = 0; c < g.Cf; c += 4) {
        const float4 v = ldq(fp + c);
        acc = fma4(ld4(wt + (c + 0) * 4), f4(v.x), acc);
        acc = fma4(ld4(wt + (c + 1) * 4), f4(v.y), acc);
        acc = fma4(ld4(wt + (c + 2) * 4), f4(v.z), acc);
        acc = fma4(ld4(wt + (c + 3) * 4), f4(v.w), acc);
      }
    }
    for (int o = 0; o < g.Cimg; ++o) {
      const long oi = (((long)b * g.Cimg + o) * g.H0 + y) * g.W0 + x;
      out[oi] = (get(acc, o) + bias[o]) + img[oi];
    }
  }
}

// ending input gradient on the padded grid: dfeat(p)[c] = sum_t sum_o w[o][c][t] dy(p - off_t)[o], dy zero off-crop
template <typename T>
__global__ void ending_bwd_x(const float* __restrict__ dy, const float* __restrict__ w, T* __restrict__ dfeat, Img g) {
  extern __shared__ float wl[];  // [t][o][Cf]
  for (int i = threadIdx.x; i < 9 * g.Cimg * g.Cf; i += blockDim.x) {
    const int c = i % g.Cf, o = (i / g.Cf) % g.Cimg, t = i / (g.Cf * g.Cimg);
    wl[i] = w[((long)o * g.Cf + c) * 9 + t];
  }
  __syncthreads();
  const int Q = g.Cf / 4;
  const long total = (long)g.B * g.Hp * g.Wp * Q;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int q = e % Q;
    const long p = e / Q;
    const int x = p % g.Wp, y = (p / g.Wp) % g.Hp, b = p / ((long)g.Wp * g.Hp);
    float4 acc = f4(0.f);
    for (int t = 0; t < 9; ++t) {
      const int yo = y - (t / 3 - 1), xo = x - (t % 3 - 1);
      if (yo < 0 || yo >= g.H0 || xo < 0 || xo >= g.W0) continue;
      for (int o = 0; o < g.Cimg; ++o) {
        const float d = dy[(((long)b * g.Cimg + o) * g.H0 + yo) * g.W0 + xo];
        acc = fma4(ld4(wl + (t * g.Cimg + o) * g.Cf + q * 4), f4(d), acc);
      }
    }
    stq(dfeat + p * g.Cf + q * 4, acc);
  }
}

// ending weight gradient: slab_w[blk][CI][Cf][9], slab_b[blk][CI]
template <int CI, typename T>
__global__ __launch_bounds__(256) void ending_bwd_w(const float* __restrict__ dy, const T* __restrict__ feat, float* __restrict__ slab_w,
                             float* __restrict__ slab_b, Img g, long px_per_blk) {
  extern __shared__ float red[];  // [blockDim][4]
  const int Q = g.Cf / 4;
  const int tid = threadIdx.x, q = tid % Q, pl = tid / Q, PPI = blockDim.x / Q;
  float4 acc[CI][9];
  float bacc[CI];
#pragma unroll
  for (int o = 0; o < CI; ++o) {
    bacc[o] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[o][t] = f4(0.f);
  }
  const long total = (long)g.B * g.H0 * g.W0;
  const long p0 = blockIdx.x * px_per_blk, p1 = min(total, p0 + px_per_blk);
  if (pl < PPI) {
    for (long p = p0 + pl; p < p1; p += PPI) {
      const int x = p % g.W0, y = (p / g.W0) % g.H0, b = p / ((long)g.W0 * g.H0);
      float d[CI];
#pragma unroll
      for (int o = 0; o < CI; ++o) {
        d[o] = dy[(((long)b * CI + o) * g.H0 + y) * g.W0 + x];
        bacc[o] += d[o];
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        if (yy < 0 || yy >= g.Hp || xx < 0 || xx >= g.Wp) continue;
        const float4 v = ldq(feat + (((long)b * g.Hp + yy) * g.Wp + xx) * g.Cf + q * 4);
#pragma unroll
        for (int o = 0; o < CI; ++o) acc[o][t] = fma4(v, f4(d[o]), acc[o][t]);
      }
    }
  }
  float* dw = slab_w + (long)blockIdx.x * CI * g.Cf * 9;
#pragma unroll
  for (int o = 0; o < CI; ++o) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      st4(red + tid * 4, acc[o][t]);
      __syncthreads();
      if (pl == 0) {
        float4 s4 = f4(0.f);
        for (int i = 0; i < PPI; ++i) s4 += ld4(red + (i * Q + q) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) dw[((long)o * g.Cf + q * 4 + j) * 9 + t] = get(s4, j);
      }
      __syncthreads();
    }
  }
  // bias: lanes with q == 0 hold the pixel-lane sums of every output channel
#pragma unroll
  for (int o = 0; o < CI; ++o) {
    red[tid] = (q == 0 && pl < PPI) ? bacc[o] : 0.f;
    __syncthreads();
    if (tid == 0) {
      float s1 = 0.f;
      for (int i = 0; i < PPI; ++i) s1 += red[i * Q];
      slab_b[(long)blockIdx.x * CI + o] = s1;
    }
    __syncthreads();
  }
}

#define NBP_DISPATCH_CI(ci, ...)                        \
  switch (ci) {                                          \
    case 1: { constexpr int CI = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int CI = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int CI = 3; __VA_ARGS__; } break; \
    default: { constexpr int CI = 4; __VA_ARGS__; } break; \
  }

int blocks_for(long total, long want_px) {
  long g = (total + want_px - 1) / want_px;
  if (g > 1024) g = 1024;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

int nbp_intro_fwd(const float* img, const float* w, const float* bias, void* out, int B, int Cimg, int H0, int W0,
                  int Hp, int Wp, int Cf, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(img && w && bias && out && B > 0 && Cimg > 0 && Cimg <= kMaxCin && Cf % 4 == 0, "nbp_intro_fwd: bad args");
  NBP_REQUIRE(Hp >= H0 && Wp >= W0, "nbp_intro_fwd: padded grid smaller than image");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long total = (long)B * Hp * Wp;
  long grid = (total + 255) / 256;
  const int gr = (int)(grid > 4096 ? 4096 : grid);
  NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, intro_fwd<CI, T><<<gr, 256, Cf * Cimg * 9 * sizeof(float), S(s)>>>(
                                                  img, w, bias, (T*)out, g)));
  return check_launch("intro_fwd");
}

size_t nbp_intro_bwd_workspace_floats(int B, int Cimg, int Hp, int Wp, int Cf) {
  return (size_t)blocks_for((long)B * Hp * Wp, 1024) * Cf * (Cimg * 9 + 1);
}

int nbp_intro_bwd(const float* img, const void* dout, const float* w, float* dw, float* db, float* dimg, float* ws,
                  int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(img && dout && w && dw && db && ws && Cimg <= kMaxCin && Cf % 4 == 0 && Cf / 4 <= 256,
              "nbp_intro_bwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long total = (long)B * Hp * Wp;
  const int nb = blocks_for(total, 1024);
  const long ppb = (total + nb - 1) / nb;
  float* slab_w = ws;
  float* slab_b = ws + (long)nb * Cf * Cimg * 9;
  NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, intro_bwd_w<CI, T><<<nb, 256, 256 * 4 * sizeof(float), S(s)>>>(
                                                  img, (const T*)dout, slab_w, slab_b, g, ppb)));
  int rc = check_launch("intro_bwd_w");
  if (rc) return rc;
  rc = nbp_reduce_slab(slab_w, nb, (long)Cf * Cimg * 9, dw, s);
  if (rc) return rc;
  rc = nbp_reduce_slab(slab_b, nb, Cf, db, s);
  if (rc) return rc;
  if (dimg) {
    const long ti = (long)B * Cimg * H0 * W0;
    long gr = (ti + 255) / 256;
    const int gx = (int)(gr > 4096 ? 4096 : gr);
    NBP_DISPATCH_T(dtype, intro_bwd_x<T><<<gx, 256, 0, S(s)>>>((const T*)dout, w, dimg, g));
  }
  return check_launch("intro_bwd");
}

int nbp_ending_fwd(const void* feat, const float* w, const float* bias, const float* img, float* out, int B, int Cimg,
                   int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(feat && w && bias && img && out && Cimg > 0 && Cimg <= kMaxCin && Cf % 4 == 0, "nbp_ending_fwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long total = (long)B * H0 * W0;
  long grid = (total + 255) / 256;
  const int gr = (int)(grid > 4096 ? 4096 : grid);
  NBP_DISPATCH_T(dtype, ending_fwd<T><<<gr, 256, 9 * Cf * 4 * sizeof(float), S(s)>>>((const T*)feat, w, bias, img, out, g));
  return check_launch("ending_fwd");
}

size_t nbp_ending_bwd_workspace_floats(int B, int Cimg, int H0, int W0, int Cf) {
  return (size_t)blocks_for((long)B * H0 * W0, 1024) * ((size_t)Cimg * Cf * 9 + Cimg);
}

int nbp_ending_bwd(const float* dy, const void* feat, const float* w, void* dfeat, float* dw, float* db, float* ws,
                   int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dy && feat && w && dfeat && dw && db && ws && Cimg <= kMaxCin && Cf % 4 == 0 && Cf / 4 <= 256,
              "nbp_ending_bwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long tx = (long)B * Hp * Wp * (Cf / 4);
  long gx = (tx + 255) / 256;
  const int gxx = (int)(gx > 4096 ? 4096 : gx);
  NBP_DISPATCH_T(dtype, ending_bwd_x<T><<<gxx, 256, 9 * Cimg * Cf * sizeof(float), S(s)>>>(dy, w, (T*)dfeat, g));
  const long total = (long)B * H0 * W0;
  const int nb = blocks_for(total, 1024);
  const long ppb = (total + nb - 1) / nb;
  float* slab_w = ws;
  float* slab_b = ws + (long)nb * Cimg * Cf * 9;
  NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, ending_bwd_w<CI, T><<<nb, 256, 256 * 4 * sizeof(float), S(s)>>>(
                                                  dy, (const T*)feat, slab_w, slab_b, g, ppb)));
  int rc = check_launch("ending_bwd_w");
  if (rc) return rc;
  rc = nbp_reduce_slab(slab_w, nb, (long)Cimg * Cf * 9, dw, s);
  if (rc) return rc;
  return nbp_reduce_slab(slab_b, nb, Cimg, db, s);
}

}  // extern "C"
