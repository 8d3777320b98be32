// NAFNet image-boundary convolutions (NAFNet_arch.py:88-91,134-136,152-162):
//   intro : 3x3 pad 1, img_channel -> width, on the input zero-padded to a multiple of 2^len(enc) (check_image_size);
//           reads the NCHW image, writes NHWC features on the padded grid.
//   ending: 3x3 pad 1, width -> img_channel on the padded grid, + global residual, cropped to the input size;
//           reads NHWC features, writes the NCHW image.
#include "nbp_common.h"

using namespace nbp;

namespace {

constexpr int kMaxCin = 4;

struct Img {
  int B, Cimg, H0, W0;  // image (unpadded)
  int Hp, Wp;           // padded feature grid
  int Cf;               // feature channels (width)
};

// ------------------------------------------------------------------ intro forward
__global__ void intro_fwd(const float* __restrict__ img, const float* __restrict__ w, const float* __restrict__ bias,
                          float* __restrict__ out, Img g) {
  extern __shared__ float wl[];  // [Cf][Cimg*9]
  const int K = g.Cimg * 9;
  for (int i = threadIdx.x; i < g.Cf * K; i += blockDim.x) wl[i] = w[i];
  __syncthreads();
  const long total = (long)g.B * g.Hp * g.Wp;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const int x = p % g.Wp, y = (p / g.Wp) % g.Hp, b = p / ((long)g.Wp * g.Hp);
    float in[kMaxCin * 9];
#pragma unroll
    for (int c = 0; c < kMaxCin; ++c) {
      if (c >= g.Cimg) break;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        in[c * 9 + t] = (yy >= 0 && yy < g.H0 && xx >= 0 && xx < g.W0)
                            ? img[(((long)b * g.Cimg + c) * g.H0 + yy) * g.W0 + xx] : 0.f;
      }
    }
    float* op = out + p * g.Cf;
    for (int o = 0; o < g.Cf; o += 4) {
      float r[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float a = bias[o + j];
        const float* wr = wl + (o + j) * K;
        for (int k = 0; k < K; ++k) a = fmaf(wr[k], in[k], a);
        r[j] = a;
      }
      st4(op + o, make_float4(r[0], r[1], r[2], r[3]));
    }
  }
}

// intro weight gradient: slab[blk][Cf][Cimg*9 + 1] (last column = bias)
__global__ void intro_bwd_w(const float* __restrict__ img, const float* __restrict__ dout, float* __restrict__ slab,
                            Img g, long px_per_blk) {
  extern __shared__ float red[];  // [blockDim][4]
  const int Q = g.Cf / 4;
  const int tid = threadIdx.x, q = tid % Q, pl = tid / Q, PPI = blockDim.x / Q;
  const int K = g.Cimg * 9;
  float4 acc[kMaxCin * 9 + 1];
#pragma unroll
  for (int k = 0; k < kMaxCin * 9 + 1; ++k) acc[k] = f4(0.f);
  const long total = (long)g.B * g.Hp * g.Wp;
  const long p0 = blockIdx.x * px_per_blk, p1 = min(total, p0 + px_per_blk);
  if (pl < PPI) {
    for (long p = p0 + pl; p < p1; p += PPI) {
      const int x = p % g.Wp, y = (p / g.Wp) % g.Hp, b = p / ((long)g.Wp * g.Hp);
      const float4 d = ld4(dout + p * g.Cf + q * 4);
      acc[kMaxCin * 9] += d;
#pragma unroll
      for (int c = 0; c < kMaxCin; ++c) {
        if (c >= g.Cimg) break;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
          const float v = (yy >= 0 && yy < g.H0 && xx >= 0 && xx < g.W0)
                              ? img[(((long)b * g.Cimg + c) * g.H0 + yy) * g.W0 + xx] : 0.f;
          acc[c * 9 + t] = fma4(d, f4(v), acc[c * 9 + t]);
        }
      }
    }
  }
  float* dst = slab + (long)blockIdx.x * g.Cf * (K + 1);
#pragma unroll
  for (int kk = 0; kk < kMaxCin * 9 + 1; ++kk) {
    if (kk >= K && kk != kMaxCin * 9) continue;  // uniform across the block
    const int col = kk == kMaxCin * 9 ? K : kk;
    st4(red + tid * 4, acc[kk]);
    __syncthreads();
    if (pl == 0) {
      float4 s = f4(0.f);
      for (int i = 0; i < PPI; ++i) s += ld4(red + (i * Q + q) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[(long)(q * 4 + j) * (K + 1) + col] = get(s, j);
    }
    __syncthreads();
  }
}

// intro input gradient (only when the image requires grad): d img = conv^T over the padded grid, restricted to H0 x W0
__global__ void intro_bwd_x(const float* __restrict__ dout, const float* __restrict__ w, float* __restrict__ dimg, Img g) {
  const long total = (long)g.B * g.Cimg * g.H0 * g.W0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = i % g.W0, y = (i / g.W0) % g.H0;
    const int c = (i / ((long)g.W0 * g.H0)) % g.Cimg;
    const int b = i / ((long)g.W0 * g.H0 * g.Cimg);
    float a = 0.f;
    for (int t = 0; t < 9; ++t) {
      const int yo = y - (t / 3 - 1), xo = x - (t % 3 - 1);
      if (yo < 0 || yo >= g.Hp || xo < 0 || xo >= g.Wp) continue;
      const float* dp = dout + (((long)b * g.Hp + yo) * g.Wp + xo) * g.Cf;
      for (int o = 0; o < g.Cf; ++o) a = fmaf(w[((long)o * g.Cimg + c) * 9 + t], dp[o], a);
    }
    dimg[i] = a;
  }
}

// ------------------------------------------------------------------ ending forward
// wl layout: [t][Cf][4] with o < Cimg (<= 4) in the last dimension
__global__ void ending_fwd(const float* __restrict__ feat, const float* __restrict__ w, const float* __restrict__ bias,
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
      const float* fp = feat + (((long)b * g.Hp + yy) * g.Wp + xx) * g.Cf;
      const float* wt = wl + t * g.Cf * 4;
      for (int c = 0; c < g.Cf; c += 4) {
        const float4 v = ld4(fp + c);
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
__global__ void ending_bwd_x(const float* __restrict__ dy, const float* __restrict__ w, float* __restrict__ dfeat, Img g) {
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
    st4(dfeat + p * g.Cf + q * 4, acc);
  }
}

// ending weight gradient: slab[blk][Cimg][Cf][9] then Cimg bias entries
__global__ void ending_bwd_w(const float* __restrict__ dy, const float* __restrict__ feat, float* __restrict__ slab, Img g,
                             long px_per_blk) {
  extern __shared__ float red[];  // [blockDim][4]
  const int Q = g.Cf / 4;
  const int tid = threadIdx.x, q = tid % Q, pl = tid / Q, PPI = blockDim.x / Q;
  float4 acc[kMaxCin][9];
  float bacc[kMaxCin];
#pragma unroll
  for (int o = 0; o < kMaxCin; ++o) {
    bacc[o] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[o][t] = f4(0.f);
  }
  const long total = (long)g.B * g.H0 * g.W0;
  const long p0 = blockIdx.x * px_per_blk, p1 = min(total, p0 + px_per_blk);
  if (pl < PPI) {
    for (long p = p0 + pl; p < p1; p += PPI) {
      const int x = p % g.W0, y = (p / g.W0) % g.H0, b = p / ((long)g.W0 * g.H0);
      float d[kMaxCin];
#pragma unroll
      for (int o = 0; o < kMaxCin; ++o) {
        d[o] = o < g.Cimg ? dy[(((long)b * g.Cimg + o) * g.H0 + y) * g.W0 + x] : 0.f;
        bacc[o] += d[o];
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        if (yy < 0 || yy >= g.Hp || xx < 0 || xx >= g.Wp) continue;
        const float4 v = ld4(feat + (((long)b * g.Hp + yy) * g.Wp + xx) * g.Cf + q * 4);
#pragma unroll
        for (int o = 0; o < kMaxCin; ++o) acc[o][t] = fma4(v, f4(d[o]), acc[o][t]);
      }
    }
  }
  const long L = (long)g.Cimg * g.Cf * 9 + g.Cimg;
  float* dst = slab + (long)blockIdx.x * L;
#pragma unroll
  for (int o = 0; o < kMaxCin; ++o) {
    if (o >= g.Cimg) break;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      st4(red + tid * 4, acc[o][t]);
      __syncthreads();
      if (pl == 0) {
        float4 s = f4(0.f);
        for (int i = 0; i < PPI; ++i) s += ld4(red + (i * Q + q) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[((long)o * g.Cf + q * 4 + j) * 9 + t] = get(s, j);
      }
      __syncthreads();
    }
  }
  // bias: every thread holds the same sums for its pixel subset; reduce over pixel lanes (q == 0 lanes only)
#pragma unroll
  for (int o = 0; o < kMaxCin; ++o) {
    if (o >= g.Cimg) break;
    red[tid] = (q == 0 && pl < PPI) ? bacc[o] : 0.f;
    __syncthreads();
    if (tid == 0) {
      float s = 0.f;
      for (int i = 0; i < PPI; ++i) s += red[i * Q];
      dst[(long)g.Cimg * g.Cf * 9 + o] = s;
    }
    __syncthreads();
  }
}

__global__ void fold_slab_2(const float* __restrict__ slab, int S_, int rows, int cols, float* __restrict__ w,
                            float* __restrict__ b, int wcols) {
  // slab rows of (cols) floats: the first wcols go to w[row][..], column wcols goes to b[row]  (intro layout)
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * cols) return;
  float s = 0.f;
  for (int k = 0; k < S_; ++k) s += slab[(long)k * rows * cols + e];
  const int r = e / cols, c = e % cols;
  if (c < wcols) w[(long)r * wcols + c] = s;
  else b[r] = s;
}

__global__ void fold_slab_flat(const float* __restrict__ slab, int S_, long L, long nw, float* __restrict__ w,
                               float* __restrict__ b) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < L; e += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < S_; ++k) s += slab[(long)k * L + e];
    if (e < nw) w[e] = s;
    else b[e - nw] = s;
  }
}

int blocks_for(long total, long want_px) {
  long g = (total + want_px - 1) / want_px;
  if (g > 1024) g = 1024;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

int nbp_intro_fwd(const float* img, const float* w, const float* bias, float* out, int B, int Cimg, int H0, int W0,
                  int Hp, int Wp, int Cf, nbp_stream_t s) {
  NBP_REQUIRE(img && w && bias && out && B > 0 && Cimg > 0 && Cimg <= kMaxCin && Cf % 4 == 0, "nbp_intro_fwd: bad args");
  NBP_REQUIRE(Hp >= H0 && Wp >= W0, "nbp_intro_fwd: padded grid smaller than image");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long total = (long)B * Hp * Wp;
  long grid = (total + 255) / 256;
  intro_fwd<<<(int)(grid > 4096 ? 4096 : grid), 256, Cf * Cimg * 9 * sizeof(float), S(s)>>>(img, w, bias, out, g);
  return check_launch("intro_fwd");
}

size_t nbp_intro_bwd_workspace_floats(int B, int Cimg, int Hp, int Wp, int Cf) {
  return (size_t)blocks_for((long)B * Hp * Wp, 1024) * Cf * (Cimg * 9 + 1);
}

int nbp_intro_bwd(const float* img, const float* dout, const float* w, float* dw, float* db, float* dimg, float* ws,
                  int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, nbp_stream_t s) {
  NBP_REQUIRE(img && dout && w && dw && db && ws && Cimg <= kMaxCin && Cf % 4 == 0 && Cf / 4 <= 256,
              "nbp_intro_bwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long total = (long)B * Hp * Wp;
  const int nb = blocks_for(total, 1024);
  const long ppb = (total + nb - 1) / nb;
  intro_bwd_w<<<nb, 256, 256 * 4 * sizeof(float), S(s)>>>(img, dout, ws, g, ppb);
  const int cols = Cimg * 9 + 1;
  fold_slab_2<<<cdiv(Cf * cols, 256), 256, 0, S(s)>>>(ws, nb, Cf, cols, dw, db, Cimg * 9);
  if (dimg) {
    const long ti = (long)B * Cimg * H0 * W0;
    long gr = (ti + 255) / 256;
    intro_bwd_x<<<(int)(gr > 4096 ? 4096 : gr), 256, 0, S(s)>>>(dout, w, dimg, g);
  }
  return check_launch("intro_bwd");
}

int nbp_ending_fwd(const float* feat, const float* w, const float* bias, const float* img, float* out, int B, int Cimg,
                   int H0, int W0, int Hp, int Wp, int Cf, nbp_stream_t s) {
  NBP_REQUIRE(feat && w && bias && img && out && Cimg > 0 && Cimg <= kMaxCin && Cf % 4 == 0, "nbp_ending_fwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long total = (long)B * H0 * W0;
  long grid = (total + 255) / 256;
  ending_fwd<<<(int)(grid > 4096 ? 4096 : grid), 256, 9 * Cf * 4 * sizeof(float), S(s)>>>(feat, w, bias, img, out, g);
  return check_launch("ending_fwd");
}

size_t nbp_ending_bwd_workspace_floats(int B, int Cimg, int H0, int W0, int Cf) {
  return (size_t)blocks_for((long)B * H0 * W0, 1024) * ((size_t)Cimg * Cf * 9 + Cimg);
}

int nbp_ending_bwd(const float* dy, const float* feat, const float* w, float* dfeat, float* dw, float* db, float* ws,
                   int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, nbp_stream_t s) {
  NBP_REQUIRE(dy && feat && w && dfeat && dw && db && ws && Cimg <= kMaxCin && Cf % 4 == 0 && Cf / 4 <= 256,
              "nbp_ending_bwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long tx = (long)B * Hp * Wp * (Cf / 4);
  long gx = (tx + 255) / 256;
  ending_bwd_x<<<(int)(gx > 4096 ? 4096 : gx), 256, 9 * Cimg * Cf * sizeof(float), S(s)>>>(dy, w, dfeat, g);
  const long total = (long)B * H0 * W0;
  const int nb = blocks_for(total, 1024);
  const long ppb = (total + nb - 1) / nb;
  ending_bwd_w<<<nb, 256, 256 * 4 * sizeof(float), S(s)>>>(dy, feat, ws, g, ppb);
  const long L = (long)Cimg * Cf * 9 + Cimg;
  fold_slab_flat<<<cdiv(L, 256), 256, 0, S(s)>>>(ws, nb, L, (long)Cimg * Cf * 9, dw, db);
  return check_launch("ending_bwd");
}

}  // extern "C"
