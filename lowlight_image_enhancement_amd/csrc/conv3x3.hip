// NAFNet image-boundary convolutions (NAFNet_arch.py:88-91,134-136,152-162):
//   intro : 3x3 pad 1, img_channel -> width, on the input zero-padded to a multiple of 2^len(enc) (check_image_size);
//           reads the NCHW image, writes NHWC features on the padded grid.
//   ending: 3x3 pad 1, width -> img_channel on the padded grid, + global residual, cropped to the input size;
//           reads NHWC features, writes the NCHW image.
#include <algorithm>

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


// ------------------------------------------------------------------ thread-per-pixel kernels, width templated
// One workgroup per feature row; each lane owns one pixel and all of its channels.  The weights are wave-uniform
// (indices are compile-time after unrolling), so they are read through the scalar cache into SGPRs: no LDS, no
// broadcast reads, one FMA per weight use.  Rows are decoded once per workgroup (32-bit), not per pixel.
template <typename T, int CF>
__device__ __forceinline__ void store_row(T* __restrict__ op, const float (&a)[CF]) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int c = 0; c < CF; c += 8) {
      vec_t<T, 8> v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (T)a[c + j];
      *reinterpret_cast<vec_t<T, 8>*>(op + c) = v;
    }
  } else {
#pragma unroll
    for (int c = 0; c < CF; c += 4) st4(reinterpret_cast<float*>(op) + c, make_float4(a[c], a[c + 1], a[c + 2], a[c + 3]));
  }
}

template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const vec_t<T, 8> b = *reinterpret_cast<const vec_t<T, 8>*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)b[j];
  } else {
    const float4 a = ld4(reinterpret_cast<const float*>(p)), b = ld4(reinterpret_cast<const float*>(p) + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}

// intro forward on MFMA: out[px][o] = sum_k patch[px][k] W[o][k] with k = c*9 + t, plus k = 9*CI -> 1 x bias[o].
// v_mfma_f32_32x32x2f32 (fp32 in / out, exact fp32 products): a wave computes 32 pixels x 32 channels per tile in
// (9*CI + 1)/2 rounded-up MFMAs; lane l supplies patch(px = l%32, k = 2s + l/32) (gathered image taps) and keeps
// W[o = l%32][k = 2s + l/32] in VGPRs.  Tiles go through LDS to leave as 16-byte row vectors.
template <int CI, typename T>
__global__ __launch_bounds__(256) void intro_fwd_mfma(const float* __restrict__ img, const float* __restrict__ w,
                                                      const float* __restrict__ bias, T* __restrict__ out, Img g) {
  constexpr int K = CI * 9, NS = (K + 2) / 2;
  __shared__ float tile[4][32][33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, li = lane & 31;
  const int row = blockIdx.x, y = row % g.Hp, b = row / g.Hp;
  const int ntiles = (g.Wp + 31) >> 5;
  int tc[NS], tdy[NS], tdx[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int k = 2 * s + half;
    tc[s] = k / 9;
    tdy[s] = (k % 9) / 3 - 1;
    tdx[s] = (k % 9) % 3 - 1;
  }
  for (int oc = 0; oc < g.Cf; oc += 32) {
    const int o = oc + li;
    float wb[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int k = 2 * s + half;
      wb[s] = o < g.Cf ? (k < K ? w[(long)o * K + k] : (k == K ? bias[o] : 0.f)) : 0.f;
    }
    const int cw = min(32, g.Cf - oc);  // channels of this chunk
    for (int tix = wave; tix < ntiles; tix += 4) {
      const int x = tix * 32 + li;
      float pa[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int k = 2 * s + half;
        const int yy = y + tdy[s], xx = x + tdx[s];
        if (k < K) {
          pa[s] = (x < g.Wp && yy >= 0 && yy < g.H0 && xx >= 0 && xx < g.W0)
                      ? img[(((long)b * CI + tc[s]) * g.H0 + yy) * g.W0 + xx] : 0.f;
        } else {
          pa[s] = k == K ? 1.f : 0.f;
        }
      }
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int s = 0; s < NS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[s], wb[s], acc, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) tile[wave][8 * (r >> 2) + 4 * half + (r & 3)][li] = acc[r];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int c8 = cw >> 3;  // 8-channel chunks per pixel in this tile
      for (int e = lane; e < 32 * c8; e += 64) {
        const int px = e / c8, ch = (e % c8) * 8, xo = tix * 32 + px;
        if (xo >= g.Wp) continue;
        T* op = out + ((long)row * g.Wp + xo) * g.Cf + oc + ch;
        const float* tp = &tile[wave][px][ch];
        if constexpr (sizeof(T) == 2) {
          vec_t<T, 8> v;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (T)tp[j];
          *reinterpret_cast<vec_t<T, 8>*>(op) = v;
        } else {
          st4(reinterpret_cast<float*>(op), make_float4(tp[0], tp[1], tp[2], tp[3]));
          st4(reinterpret_cast<float*>(op) + 4, make_float4(tp[4], tp[5], tp[6], tp[7]));
        }
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

// ending forward on the crop: out[b][o][y][x] = (sum_t sum_c w[o][c][t] feat(y+dy, x+dx)[c] + bias[o]) + img
template <int CI, int CF, typename T>
__global__ __launch_bounds__(256) void ending_fwd_px(const T* __restrict__ feat, const float* __restrict__ w,
                                                     const float* __restrict__ bias, const float* __restrict__ img,
                                                     float* __restrict__ out, Img g) {
  const int row = blockIdx.x, y = row % g.H0, b = row / g.H0;
  for (int x = threadIdx.x; x < g.W0; x += blockDim.x) {
    float acc[CI];
#pragma unroll
    for (int o = 0; o < CI; ++o) acc[o] = 0.f;
    auto tap = [&](int t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if (yy < 0 || yy >= g.Hp || xx < 0 || xx >= g.Wp) return;
      const T* fp = feat + (((long)b * g.Hp + yy) * g.Wp + xx) * CF;
#pragma unroll
      for (int c = 0; c < CF; c += 8) {
        float v[8];
        load8(fp + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int o = 0; o < CI; ++o) acc[o] = fmaf(w[(o * CF + c + j) * 9 + t], v[j], acc[o]);
      }
    };
    if constexpr (CF >= 64) {
      // the tap loop stays rolled at 64 channels: unrolled, its 9 x 64 x CI FMAs with their scalar weight loads
      // outgrow the instruction cache (300 us per launch at w64 against 56 at w32)
#pragma unroll 1
      for (int t = 0; t < 9; ++t) tap(t);
    } else {
#pragma unroll
      for (int t = 0; t < 9; ++t) tap(t);
    }
#pragma unroll
    for (int o = 0; o < CI; ++o) {
      const long oi = (((long)b * CI + o) * g.H0 + y) * g.W0 + x;
      out[oi] = (acc[o] + bias[o]) + img[oi];
    }
  }
}

// ending input gradient on the padded grid (dy is zero off the crop).  Weights in LDS as [t][o][CF] rows (broadcast
// ds_read_b128, not SGPR re-fetches), the lane's CF accumulators as packed channel pairs; per channel the FMAs run in
// the order t, o of the scalar form.
template <int CI, int CF, typename T>
__global__ __launch_bounds__(256) void ending_bwd_x_px(const float* __restrict__ dy, const float* __restrict__ w,
                                                       T* __restrict__ dfeat, Img g) {
  __shared__ __attribute__((aligned(16))) float wl[9 * CI * CF];  // [t][o][c] = w[o][c][t]
  for (int i = threadIdx.x; i < 9 * CI * CF; i += blockDim.x) {
    const int c = i % CF, o = (i / CF) % CI, t = i / (CF * CI);
    wl[i] = w[(o * CF + c) * 9 + t];
  }
  __syncthreads();
  const int row = blockIdx.x, y = row % g.Hp, b = row / g.Hp;
  for (int x = threadIdx.x; x < g.Wp; x += blockDim.x) {
    f2v acc[CF / 2];
#pragma unroll
    for (int c = 0; c < CF / 2; ++c) acc[c] = f2v{0.f, 0.f};
#pragma unroll 1
    for (int t = 0; t < 9; ++t) {
      const int yo = y - (t / 3 - 1), xo = x - (t % 3 - 1);
      if (yo < 0 || yo >= g.H0 || xo < 0 || xo >= g.W0) continue;
#pragma unroll
      for (int o = 0; o < CI; ++o) {
        const float d = dy[(((long)b * CI + o) * g.H0 + yo) * g.W0 + xo];
        const f2v dd = f2v{d, d};
        const float4* wr = reinterpret_cast<const float4*>(wl + (t * CI + o) * CF);
#pragma unroll
        for (int c4 = 0; c4 < CF / 4; ++c4) {
          const float4 wq = wr[c4];
          acc[2 * c4] = __builtin_elementwise_fma(f2v{wq.x, wq.y}, dd, acc[2 * c4]);
          acc[2 * c4 + 1] = __builtin_elementwise_fma(f2v{wq.z, wq.w}, dd, acc[2 * c4 + 1]);
        }
      }
    }
    float a[CF];
#pragma unroll
    for (int c = 0; c < CF / 2; ++c) {
      a[2 * c] = acc[c].x;
      a[2 * c + 1] = acc[c].y;
    }
    store_row<T, CF>(dfeat + ((long)row * g.Wp + x) * CF, a);
  }
}

// ------------------------------------------------------------------ boundary-conv weight gradients on MFMA
// D[m][n] = sum_px A(m, px) B(px, n) with v_mfma_f32_32x32x2f32: one MFMA per pixel pair (lane l supplies
// A(m = l%32, px = 2i + l/32) and B(px = 2i + l/32, n = l%32)), fp32 operands and accumulation.
//   MODE 0 (intro):  m = output channel o, A = dout[px][o]; n = c*9 + t -> image tap, n == 9*CI -> 1 (bias column)
//   MODE 1 (ending): m = feature channel c, A = feat[px][c]; n = o*9 + t -> dy[o] at px - tap offset (0 off-crop);
//                    db[o] = sum of the centre-tap column (n = o*9 + 4), accumulated beside the MFMA
// Grid (blocks over feature rows, M chunks of 32, N chunks of 32); block x writes slab x (fixed-order reductions).
template <int MODE, int CI, typename T>
__global__ __launch_bounds__(256) void bconv_wgrad(const float* __restrict__ src, const T* __restrict__ nhwc,
                                                   float* __restrict__ slab_w, float* __restrict__ slab_b, Img g) {
  __shared__ float red[4][32][33];
  __shared__ float bred[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5;
  const int m = blockIdx.y * 32 + (lane & 31), n = blockIdx.z * 32 + (lane & 31);
  constexpr int NK = 9 * CI;
  const int nc = n / 9, nt = n % 9, ndy = nt / 3 - 1, ndx = nt % 3 - 1;
  const bool mval = m < g.Cf;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float bacc = 0.f;
  const int rows = g.B * g.Hp, pairs = (g.Wp + 1) >> 1;
  // U pixel pairs per step: all 2U operand loads are issued before the MFMAs that consume them (latency hiding)
  constexpr int U = 8;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int y = row % g.Hp, b = row / g.Hp;
    const T* arow = nhwc + (long)row * g.Wp * g.Cf;
    for (int i0 = wave; i0 < pairs; i0 += 4 * U) {
      float av[U], bv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int x = 2 * (i0 + 4 * u) + half;
        const bool xval = x < g.Wp;
        av[u] = (mval && xval) ? (float)arow[(long)x * g.Cf + m] : 0.f;
        bv[u] = 0.f;
        if (MODE == 0) {
          const int yy = y + ndy, xx = x + ndx;
          if (n < NK) {
            if (xval && yy >= 0 && yy < g.H0 && xx >= 0 && xx < g.W0)
              bv[u] = src[(((long)b * CI + nc) * g.H0 + yy) * g.W0 + xx];
          } else if (n == NK) {
            bv[u] = xval ? 1.f : 0.f;
          }
        } else {
          const int yo = y - ndy, xo = x - ndx;
          if (n < NK && xval && yo >= 0 && yo < g.H0 && xo >= 0 && xo < g.W0)
            bv[u] = src[(((long)b * CI + nc) * g.H0 + yo) * g.W0 + xo];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (MODE == 1 && nt == 4) bacc += bv[u];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][8 * (r >> 2) + 4 * half + (r & 3)][lane & 31] = acc[r];
  if (MODE == 1) bred[wave][lane] = bacc;
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += 256) {
    const int mi = e >> 5, ni = e & 31;
    const int mm = blockIdx.y * 32 + mi, nn = blockIdx.z * 32 + ni;
    const float v = ((red[0][mi][ni] + red[1][mi][ni]) + red[2][mi][ni]) + red[3][mi][ni];
    if (mm >= g.Cf) continue;
    if (MODE == 0) {
      if (nn < NK) slab_w[((long)blockIdx.x * g.Cf + mm) * NK + nn] = v;
      else if (nn == NK) slab_b[(long)blockIdx.x * g.Cf + mm] = v;
    } else if (nn < NK) {
      slab_w[(long)blockIdx.x * CI * g.Cf * 9 + ((long)(nn / 9) * g.Cf + mm) * 9 + nn % 9] = v;
    }
  }
  if (MODE == 1 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x < CI) {
    const int l = threadIdx.x * 9 + 4;  // lane of column o*9+4 (< 32 for CI <= 4), both half-waves
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += bred[w][l] + bred[w][l + 32];
    slab_b[(long)blockIdx.x * CI + threadIdx.x] = s;
  }
}

// Same contraction, operands staged through LDS: per (feature row, chunk of XC pixels) the block's 32 feature
// channels (16-byte coalesced loads, XC * 64 B) and the three source rows around the feature row (CI planes, XC + 2
// columns with zero padding) -- the gather above issues one 64-lane scattered load per MFMA operand.  The next
// chunk's operands are loaded into registers while the MFMAs consume the current one.  Each wave runs the same
// pixel-pair sequence (i = wave, wave + 4, ...) as the gather kernel, so every slab is bitwise the same.  Needs Cf a
// multiple of 16 / sizeof(T).
template <int MODE, int CI, typename T>
__global__ __launch_bounds__(256, 4) void bconv_wgrad_lds(const float* __restrict__ src, const T* __restrict__ nhwc,
                                                       float* __restrict__ slab_w, float* __restrict__ slab_b, Img g) {
  constexpr int XC = 512 / sizeof(T);           // pixels per chunk: 16 KB of feature operand
  constexpr int PPX = 32 * sizeof(T) / 16;      // 16-byte pieces per pixel
  constexpr int EPP = 16 / sizeof(T);           // elements per piece
  constexpr int BW = XC + 2;                    // staged source columns (x0 - 1 .. x0 + XC)
  static_assert((XC / 2) % 4 == 0, "each wave keeps its pair residue across chunks");
  // the operand tiles and the final cross-wave reduction share one LDS buffer (26 KB)
  // bs rows: CI * 3 source rows, then a row of ones (the bias column's operand) and a row of zeros (columns past NK)
  constexpr int AS_B = XC * 32 * (int)sizeof(T), BS_B = (CI * 3 + 2) * BW * 4, RED_B = 4 * 32 * 33 * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[(AS_B + BS_B > RED_B) ? AS_B + BS_B : RED_B];
  __shared__ float bred[4][64];
  auto as = reinterpret_cast<T (*)[32]>(smem);
  auto bs = reinterpret_cast<float (*)[3][BW]>(smem + AS_B);
  auto red = reinterpret_cast<float (*)[32][33]>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, half = lane >> 5;
  const int m0 = blockIdx.y * 32;
  const int n = blockIdx.z * 32 + (lane & 31);
  constexpr int NK = 9 * CI;
  const int nc = n / 9, nt = n % 9, ndy = nt / 3 - 1, ndx = nt % 3 - 1;
  // this lane's source tap relative to the chunk's staged rows / columns
  const int ky = MODE == 0 ? ndy + 1 : 1 - ndy, kx = MODE == 0 ? ndx + 1 : 1 - ndx;
  const bool ntap = n < NK, nbias = MODE == 0 && n == NK;
  const int bc = ntap ? nc : 0;
  // full chunks: this lane's operand addresses advance by a pair per MFMA with no per-pixel test
  const float* bsx = &bs[0][0][0];
  const float* bp = bsx + (ntap ? (nc * 3 + ky) * BW + kx : (nbias ? CI * 3 : CI * 3 + 1) * BW + 1) + half;
  const T* ap = &as[half][lane & 31];
  const float bm = (MODE == 1 && ntap && nt == 4) ? 1.f : 0.f;
  for (int j = tid; j < 2 * BW; j += 256) (&bs[0][0][0])[CI * 3 * BW + j] = j < BW ? 1.f : 0.f;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float bacc = 0.f;
  const int rows = g.B * g.Hp;
  constexpr int KA = XC * PPX / 256, NBS = (CI * 3 * BW + 255) / 256;
  uint4 va[KA];
  float sv[NBS];
  auto load = [&](int row, int x0) {
    const int y = row % g.Hp, b = row / g.Hp;
    const T* arow = nhwc + (long)row * g.Wp * g.Cf;
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      const int q = tid + k * 256, px = q / PPX, part = q % PPX;
      const int x = x0 + px, c = m0 + part * EPP;
      va[k] = make_uint4(0u, 0u, 0u, 0u);
      if (x < g.Wp && c < g.Cf) va[k] = *reinterpret_cast<const uint4*>(arow + (long)x * g.Cf + c);
    }
#pragma unroll
    for (int u = 0; u < NBS; ++u) {
      const int e = tid + u * 256;
      const int c = e / (3 * BW), k = (e / BW) % 3, j = e % BW;
      const int yy = y + k - 1, xx = x0 - 1 + j;
      sv[u] = 0.f;
      if (e < CI * 3 * BW && yy >= 0 && yy < g.H0 && xx >= 0 && xx < g.W0)
        sv[u] = src[(((long)b * CI + c) * g.H0 + yy) * g.W0 + xx];
    }
  };
  int row = blockIdx.x, x0 = 0;
  if (row < rows) load(row, 0);
  while (row < rows) {
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      const int q = tid + k * 256;
      *reinterpret_cast<uint4*>(&as[q / PPX][(q % PPX) * EPP]) = va[k];
    }
#pragma unroll
    for (int u = 0; u < NBS; ++u) {
      const int e = tid + u * 256;
      if (e < CI * 3 * BW) (&bs[0][0][0])[e] = sv[u];
    }
    __syncthreads();
    int nrow = row, nx0 = x0 + XC;
    if (nx0 >= g.Wp) { nx0 = 0; nrow += gridDim.x; }
    if (nrow < rows) load(nrow, nx0);
    // U pairs' operands read before their MFMAs; pairs past the chunk read pair 0 and contribute zeros.  Pixels past
    // the grid have a zero feature operand (staged so), which zeroes their products whatever the source tap holds.
    const int np = min(XC, g.Wp - x0 + 1) >> 1;  // pixel pairs of this chunk (the last may hold one pixel)
    constexpr int U = 8;
    if (np == XC / 2) {
      for (int i0 = wave; i0 < XC / 2; i0 += 4 * U) {
        float av[U], bv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = i0 + 4 * u;
          av[u] = (float)ap[i * 64];
          bv[u] = bp[2 * i];
          if (MODE == 1) bacc = fmaf(bm, bv[u], bacc);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[u], bv[u], acc, 0, 0, 0);
      }
    } else {
      // the row's last, partial chunk: one pair per step (the same MFMA sequence)
      for (int i = wave; i < np; i += 4) {
        const int xl = 2 * i + half;
        const bool xval = x0 + xl < g.Wp;
        const float av = (float)as[xl][lane & 31];
        const float bt = bs[bc][ky][xl + kx];
        const float bv = ntap ? bt : ((nbias && xval) ? 1.f : 0.f);
        if (MODE == 1 && nt == 4) bacc += (ntap && xval) ? bt : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
      }
    }
    __syncthreads();
    row = nrow;
    x0 = nx0;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][8 * (r >> 2) + 4 * half + (r & 3)][lane & 31] = acc[r];
  if (MODE == 1) bred[wave][lane] = bacc;
  __syncthreads();
  for (int e = threadIdx.x; e < 32 * 32; e += 256) {
    const int mi = e >> 5, ni = e & 31;
    const int mm = blockIdx.y * 32 + mi, nn = blockIdx.z * 32 + ni;
    const float v = ((red[0][mi][ni] + red[1][mi][ni]) + red[2][mi][ni]) + red[3][mi][ni];
    if (mm >= g.Cf) continue;
    if (MODE == 0) {
      if (nn < NK) slab_w[((long)blockIdx.x * g.Cf + mm) * NK + nn] = v;
      else if (nn == NK) slab_b[(long)blockIdx.x * g.Cf + mm] = v;
    } else if (nn < NK) {
      slab_w[(long)blockIdx.x * CI * g.Cf * 9 + ((long)(nn / 9) * g.Cf + mm) * 9 + nn % 9] = v;
    }
  }
  if (MODE == 1 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x < CI) {
    const int l = threadIdx.x * 9 + 4;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) s += bred[w][l] + bred[w][l + 32];
    slab_b[(long)blockIdx.x * CI + threadIdx.x] = s;
  }
}

// NBP_BCONV_GATHER=1 (read per launch): the gather kernel -- the reference of the bitwise test
bool bconv_lds(int Cf, int esize) {
  const char* e = getenv("NBP_BCONV_GATHER");
  if (e && e[0] == '1') return false;
  return Cf % (16 / esize) == 0;
}

#define NBP_DISPATCH_CF(cf, ok, ...)                     \
  switch (cf) {                                          \
    case 8: { constexpr int CF = 8; __VA_ARGS__; } break;  \
    case 16: { constexpr int CF = 16; __VA_ARGS__; } break; \
    case 32: { constexpr int CF = 32; __VA_ARGS__; } break; \
    case 64: { constexpr int CF = 64; __VA_ARGS__; } break; \
    default: ok = false;                                 \
  }

constexpr int kWgradBlocks = 1024;

#define NBP_DISPATCH_CI(ci, ...)                        \
  switch (ci) {                                          \
    case 1: { constexpr int CI = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int CI = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int CI = 3; __VA_ARGS__; } break; \
    default: { constexpr int CI = 4; __VA_ARGS__; } break; \
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
  if (Cf % 8 == 0) {
    NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, intro_fwd_mfma<CI, T><<<B * Hp, 256, 0, S(s)>>>(img, w, bias, (T*)out, g)));
  } else {
    NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, intro_fwd<CI, T><<<gr, 256, Cf * Cimg * 9 * sizeof(float), S(s)>>>(
                                                    img, w, bias, (T*)out, g)));
  }
  return check_launch("intro_fwd");
}

size_t nbp_intro_bwd_workspace_floats(int B, int Cimg, int Hp, int Wp, int Cf) {
  (void)Wp;
  return (size_t)std::min(kWgradBlocks, B * Hp) * Cf * (Cimg * 9 + 1);
}

int nbp_intro_bwd(const float* img, const void* dout, const float* w, float* dw, float* db, float* dimg, float* ws,
                  int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(img && dout && w && dw && db && ws && Cimg <= kMaxCin && Cf % 4 == 0 && Cf / 4 <= 256,
              "nbp_intro_bwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const int nb = std::min(kWgradBlocks, B * Hp);
  float* slab_w = ws;
  float* slab_b = ws + (long)nb * Cf * Cimg * 9;
  const dim3 grid(nb, cdiv(Cf, 32), cdiv(Cimg * 9 + 1, 32));
  NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, {
    if (bconv_lds(Cf, (int)sizeof(T)))
      bconv_wgrad_lds<0, CI, T><<<grid, 256, 0, S(s)>>>(img, (const T*)dout, slab_w, slab_b, g);
    else
      bconv_wgrad<0, CI, T><<<grid, 256, 0, S(s)>>>(img, (const T*)dout, slab_w, slab_b, g);
  }));
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
  bool px = true;
  NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, NBP_DISPATCH_CF(Cf, px, ending_fwd_px<CI, CF, T><<<B * H0, 256, 0, S(s)>>>(
                                                  (const T*)feat, w, bias, img, out, g))));
  if (!px)
    NBP_DISPATCH_T(dtype, ending_fwd<T><<<gr, 256, 9 * Cf * 4 * sizeof(float), S(s)>>>((const T*)feat, w, bias, img,
                                                                                          out, g));
  return check_launch("ending_fwd");
}

size_t nbp_ending_bwd_workspace_floats(int B, int Cimg, int H0, int W0, int Cf) {
  (void)W0;
  return (size_t)std::min(kWgradBlocks, B * H0) * ((size_t)Cimg * Cf * 9 + Cimg);
}

int nbp_ending_bwd(const float* dy, const void* feat, const float* w, void* dfeat, float* dw, float* db, float* ws,
                   int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dy && feat && w && dfeat && dw && db && ws && Cimg <= kMaxCin && Cf % 4 == 0 && Cf / 4 <= 256,
              "nbp_ending_bwd: bad args");
  Img g{B, Cimg, H0, W0, Hp, Wp, Cf};
  const long tx = (long)B * Hp * Wp * (Cf / 4);
  long gx = (tx + 255) / 256;
  const int gxx = (int)(gx > 4096 ? 4096 : gx);
  bool px = true;
  NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, NBP_DISPATCH_CF(Cf, px, ending_bwd_x_px<CI, CF, T><<<B * Hp, 256, 0, S(s)>>>(
                                                  dy, w, (T*)dfeat, g))));
  if (!px)
    NBP_DISPATCH_T(dtype, ending_bwd_x<T><<<gxx, 256, 9 * Cimg * Cf * sizeof(float), S(s)>>>(dy, w, (T*)dfeat, g));
  const int nb = std::min(kWgradBlocks, B * H0);
  float* slab_w = ws;
  float* slab_b = ws + (long)nb * Cimg * Cf * 9;
  const dim3 grid(nb, cdiv(Cf, 32), cdiv(Cimg * 9, 32));
  NBP_DISPATCH_T(dtype, NBP_DISPATCH_CI(Cimg, {
    if (bconv_lds(Cf, (int)sizeof(T)))
      bconv_wgrad_lds<1, CI, T><<<grid, 256, 0, S(s)>>>(dy, (const T*)feat, slab_w, slab_b, g);
    else
      bconv_wgrad<1, CI, T><<<grid, 256, 0, S(s)>>>(dy, (const T*)feat, slab_w, slab_b, g);
  }));
  int rc = check_launch("ending_bwd_w");
  if (rc) return rc;
  rc = nbp_reduce_slab(slab_w, nb, (long)Cimg * Cf * 9, dw, s);
  if (rc) return rc;
  return nbp_reduce_slab(slab_b, nb, Cimg, db, s);
}

}  // extern "C"
