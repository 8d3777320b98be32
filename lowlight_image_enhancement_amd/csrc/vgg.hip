// VGG feature-loss glue around the implicit-GEMM 3x3 convs (nbp_conv3x3_bf16), NHWC activations stored as
// `dtype` (0 fp32: the parity mode, the reference's fp32 trunk; 1 bf16; 2 fp16):
//   PerceptualLoss (NewBP_model/losses.py:32-69): (clamp01(x) - mean) / std -> vgg19.features[:36] -> MSE / L1;
//   the LPIPS backbone taps reuse the same pieces.
// Kernels: the input prologue (NCHW fp32 -> NHWC bf16 with the channel dim padded to 8), 2x2 max-pool with argmax
// (first maximum in window order, as torch's max_pool2d) and its backward fused with the ReLU mask of the pool input,
// the feature distance with its gradient (fused with the last ReLU's mask), and the input-gradient epilogue.
#include <math.h>

#include "nbp_common.h"

using namespace nbp;

namespace {

template <typename HT>
__global__ __launch_bounds__(256) void vgg_prep_kernel(const float* __restrict__ x, long HW, long npix, int clamp,
                                                       float m0, float m1, float m2, float s0, float s1, float s2,
                                                       HT* __restrict__ y) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const float* xb = x + b * 3 * HW + q;
    float v0 = xb[0], v1 = xb[HW], v2 = xb[2 * HW];
    if (clamp) {
      v0 = fminf(fmaxf(v0, 0.f), 1.f);
      v1 = fminf(fmaxf(v1, 0.f), 1.f);
      v2 = fminf(fmaxf(v2, 0.f), 1.f);
    }
    vec_t<HT, 8> o;
    o[0] = (HT)((v0 - m0) / s0);
    o[1] = (HT)((v1 - m1) / s1);
    o[2] = (HT)((v2 - m2) / s2);
#pragma unroll
    for (int j = 3; j < 8; ++j) o[j] = (HT)0.f;
    *reinterpret_cast<vec_t<HT, 8>*>(y + p * 8) = o;
  }
}

// 2x2 / stride-2 max pool over NHWC (floor), 8 channels per thread; idx = window position 0..3 of the maximum
template <typename HT>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const HT* __restrict__ x, int H, int W, int C, long total8,
                                                          HT* __restrict__ y, unsigned char* __restrict__ idx) {
  const int Ho = H / 2, Wo = W / 2, C8 = C / 8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int c8 = e % C8;
    const long o = e / C8;  // output pixel
    const int j = o % Wo;
    const long t = o / Wo;
    const int i = t % Ho;
    const long b = t / Ho;
    const HT* base = x + (((b * H + 2 * i) * W + 2 * j) * C + c8 * 8);
    const vec_t<HT, 8> a = *reinterpret_cast<const vec_t<HT, 8>*>(base);
    const vec_t<HT, 8> bq = *reinterpret_cast<const vec_t<HT, 8>*>(base + C);
    const vec_t<HT, 8> cq = *reinterpret_cast<const vec_t<HT, 8>*>(base + (long)W * C);
    const vec_t<HT, 8> dq = *reinterpret_cast<const vec_t<HT, 8>*>(base + (long)W * C + C);
    vec_t<HT, 8> out;
    unsigned long long packed = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float best = (float)a[k];
      int bi = 0;
      const float v1 = (float)bq[k], v2 = (float)cq[k], v3 = (float)dq[k];
      if (v1 > best || v1 != v1) { best = v1; bi = 1; }
      if (v2 > best || v2 != v2) { best = v2; bi = 2; }
      if (v3 > best || v3 != v3) { best = v3; bi = 3; }
      out[k] = (HT)best;
      packed |= (unsigned long long)bi << (8 * k);
    }
    *reinterpret_cast<vec_t<HT, 8>*>(y + o * C + c8 * 8) = out;
    *reinterpret_cast<unsigned long long*>(idx + o * C + c8 * 8) = packed;
  }
}

// din = scatter(dout at the argmax) * !(post_in <= 0)   (the pool input is a post-ReLU map; torch's threshold_backward
// passes the gradient of a NaN)
template <typename HT>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const HT* __restrict__ dy,
                                                          const unsigned char* __restrict__ idx,
                                                          const HT* __restrict__ post_in, int H, int W, int C,
                                                          long total8, HT* __restrict__ dx) {
  const int Ho = H / 2, Wo = W / 2, C8 = C / 8;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int c8 = e % C8;
    const long pix = e / C8;  // input pixel
    const int j = pix % W;
    const long t = pix / W;
    const int i = t % H;
    const long b = t / H;
    vec_t<HT, 8> out;
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = (HT)0.f;
    const int io = i / 2, jo = j / 2;
    if (io < Ho && jo < Wo) {
      const long o = ((b * Ho + io) * Wo + jo) * C + c8 * 8;
      const int pos = (i & 1) * 2 + (j & 1);
      const vec_t<HT, 8> g = *reinterpret_cast<const vec_t<HT, 8>*>(dy + o);
      const unsigned long long packed = *reinterpret_cast<const unsigned long long*>(idx + o);
      const vec_t<HT, 8> pin = *reinterpret_cast<const vec_t<HT, 8>*>(post_in + pix * C + c8 * 8);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if ((int)((packed >> (8 * k)) & 0xff) == pos && !((float)pin[k] <= 0.f)) out[k] = g[k];  // relu bwd: NaN passes
    }
    *reinterpret_cast<vec_t<HT, 8>*>(dx + pix * C + c8 * 8) = out;
  }
}

// loss partials of mode 0: (a - b)^2, mode 1: |a - b|
template <typename HT>
__global__ __launch_bounds__(256) void feat_dist_fwd(const HT* __restrict__ a, const HT* __restrict__ b, long n,
                                                     int mode, double* __restrict__ part) {
  __shared__ double red[16];
  double acc = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = (float)a[i] - (float)b[i];
    acc += mode == 0 ? (double)(d * d) : (double)fabsf(d);
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void feat_dist_finalize(const double* __restrict__ part, int n, double scale, float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += part[i];
    out[0] = (float)(s * scale);
  }
}

// da = up[0] * scale * (mode 0: 2 (a - b), mode 1: sign(a - b)) * (relu_mask ? (a > 0) : 1)
template <typename HT>
__global__ __launch_bounds__(256) void feat_dist_bwd(const HT* __restrict__ a, const HT* __restrict__ b, long n,
                                                     int mode, float scale, int relu_mask, const float* __restrict__ up,
                                                     HT* __restrict__ da) {
  const float g = up[0] * scale;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float av = (float)a[i], d = av - (float)b[i];
    float v = mode == 0 ? 2.f * d : (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
    if (relu_mask && !(av > 0.f)) v = 0.f;
    da[i] = (HT)(g * v);
  }
}

// dx (NCHW fp32) = d8[..][c] / std[c] * (clamp ? (0 <= x <= 1) : 1), c < 3
__global__ __launch_bounds__(256) void vgg_input_grad_kernel(const float* __restrict__ d8, const float* __restrict__ x,
                                                             long HW, long npix, int clamp, float s0, float s1,
                                                             float s2, float* __restrict__ dx) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const float sd[3] = {s0, s1, s2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const long o = (b * 3 + c) * HW + q;
      const float xv = x[o];
      const bool pass = !clamp || (xv >= 0.f && xv <= 1.f);
      dx[o] = pass ? d8[p * 8 + c] / sd[c] : 0.f;
    }
  }
}

// d += g * (post > 0)  (a tapped post-ReLU map's gradient joining the backward walk), all bf16
template <typename HT>
__global__ __launch_bounds__(256) void add_relu_masked_kernel(HT* __restrict__ d, const HT* __restrict__ g,
                                                              const HT* __restrict__ post, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    if ((float)post[i] > 0.f) d[i] = (HT)((float)d[i] + (float)g[i]);
}

// ---------------------------------------------------------------- LPIPS tap distance (lpips 0.1.4, net='vgg')
// per pixel: u = a / (|a| + 1e-10), v = b / (|b| + 1e-10) over the C channels (normalize_tensor),
// d = sum_c w_c (u_c - v_c)^2 (the 1x1 'lin' head); per image out[n] (+)= mean over pixels (spatial_average).
// LPIPS tap (lpips 0.1.4 pretrained_networks / lpips.py: normalize_tensor over channels, (u - v)^2, 1x1 `lin` conv,
// spatial mean): a pixel's C channels are C / 8 chunks of 16 bytes spread over a group of G lanes (G a power of two,
// V chunks per lane; lanes past the last chunk masked), so every load is a coalesced row piece and the feature
// vectors are read from HBM once (kept in registers between the norm pass and the distance / gradient pass);
// channel sums are group shuffles.  Groups stride over the pixels.
template <int G, int V, typename HT>
struct TapRow {
  vec_t<HT, 8> a[V], b[V];
  bool ok[V];
};

template <int G, int V, typename HT>
__device__ __forceinline__ void tap_load(TapRow<G, V, HT>& r, const HT* pa, const HT* pb, int lg, int nch) {
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int ch = j * G + lg;
    r.ok[j] = ch < nch;
    if (r.ok[j]) {
      r.a[j] = *reinterpret_cast<const vec_t<HT, 8>*>(pa + ch * 8);
      r.b[j] = *reinterpret_cast<const vec_t<HT, 8>*>(pb + ch * 8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) r.a[j][e] = r.b[j][e] = (HT)0.f;
    }
  }
}

template <int G, int V, typename HT>
__global__ __launch_bounds__(256) void lpips_tap_fwd(const HT* __restrict__ a, const HT* __restrict__ b,
                                                     const float* __restrict__ w, long HW, int C, int chunks,
                                                     double* __restrict__ slab) {
  __shared__ double red[16];
  constexpr int GPB = 256 / G;  // pixel groups per block
  const int n = blockIdx.y, lg = threadIdx.x % G, grp = threadIdx.x / G, nch = C / 8;
  const long per = (HW + chunks - 1) / chunks, q0 = (long)blockIdx.x * per, q1 = min(HW, q0 + per);
  float wr[V][8];
#pragma unroll
  for (int j = 0; j < V; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) wr[j][e] = j * G + lg < nch ? w[(j * G + lg) * 8 + e] : 0.f;
  double acc = 0.0;
  for (long q = q0 + grp; q < q1; q += GPB) {
    TapRow<G, V, HT> r;
    tap_load<G, V, HT>(r, a + ((long)n * HW + q) * C, b + ((long)n * HW + q) * C, lg, nch);
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sa = fmaf((float)r.a[j][e], (float)r.a[j][e], sa);
        sb = fmaf((float)r.b[j][e], (float)r.b[j][e], sb);
      }
    sa = group_sum<G>(sa);
    sb = group_sum<G>(sb);
    const float ia = 1.f / (sqrtf(sa) + 1e-10f), ib = 1.f / (sqrtf(sb) + 1e-10f);
    float d = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = (float)r.a[j][e] * ia - (float)r.b[j][e] * ib;
        d = fmaf(wr[j][e] * t, t, d);
      }
    acc += (double)d;
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) slab[(long)n * chunks + blockIdx.x] = t;
}

__global__ void lpips_finalize(const double* __restrict__ slab, int N, int chunks, double inv_hw, int accumulate,
                               float* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += slab[(long)n * chunks + c];
  out[n] = (float)((accumulate ? (double)out[n] : 0.0) + s * inv_hw);
}

// d a_k = up[n] / HW * (g_k / na - a_k (sum_c g_c a_c) / (na^2 |a|)),  g_c = 2 w_c (u_c - v_c), na = |a| + 1e-10.
// A pixel whose feature vector is all zero gets zero gradient (torch's sqrt backward yields NaN there).
template <int G, int V, typename HT>
__global__ __launch_bounds__(256) void lpips_tap_bwd(const HT* __restrict__ a, const HT* __restrict__ b,
                                                     const float* __restrict__ w, long HW, int C, long npix,
                                                     const float* __restrict__ up, HT* __restrict__ da) {
  constexpr int GPB = 256 / G;
  const int lg = threadIdx.x % G, grp = threadIdx.x / G, nch = C / 8;
  float wr[V][8];
#pragma unroll
  for (int j = 0; j < V; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) wr[j][e] = j * G + lg < nch ? 2.f * w[(j * G + lg) * 8 + e] : 0.f;
  for (long p = (long)blockIdx.x * GPB + grp; p < npix; p += (long)gridDim.x * GPB) {
    const long n = p / HW;
    TapRow<G, V, HT> r;
    tap_load<G, V, HT>(r, a + p * C, b + p * C, lg, nch);
    HT* pd = da + p * C;
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sa = fmaf((float)r.a[j][e], (float)r.a[j][e], sa);
        sb = fmaf((float)r.b[j][e], (float)r.b[j][e], sb);
      }
    sa = group_sum<G>(sa);
    sb = group_sum<G>(sb);
    if (sa == 0.f) {
      vec_t<HT, 8> z;
#pragma unroll
      for (int e = 0; e < 8; ++e) z[e] = (HT)0.f;
#pragma unroll
      for (int j = 0; j < V; ++j)
        if (r.ok[j]) *reinterpret_cast<vec_t<HT, 8>*>(pd + (j * G + lg) * 8) = z;
      continue;
    }
    const float ra = sqrtf(sa), na = ra + 1e-10f, ia = 1.f / na, ib = 1.f / (sqrtf(sb) + 1e-10f);
    float gs = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float av = (float)r.a[j][e];
        gs = fmaf(wr[j][e] * (av * ia - (float)r.b[j][e] * ib), av, gs);
      }
    gs = group_sum<G>(gs);
    const float sc = up[n] / (float)HW, k2 = gs / (na * na * ra);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      if (!r.ok[j]) continue;
      vec_t<HT, 8> o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float av = (float)r.a[j][e];
        const float g = wr[j][e] * (av * ia - (float)r.b[j][e] * ib);
        o[e] = (HT)(sc * (g * ia - av * k2));
      }
      *reinterpret_cast<vec_t<HT, 8>*>(pd + (j * G + lg) * 8) = o;
    }
  }
}

// k x k max pool, stride s, no padding (floor), NHWC (torchvision AlexNet's MaxPool2d(3, 2)); idx (optional): the
// window position of the first maximum in row-major window order (a NaN replaces the running maximum, so the last NaN wins, as torch's max_pool2d)
template <typename HT>
__global__ __launch_bounds__(256) void maxpool_k_fwd_kernel(const HT* __restrict__ x, int H, int W, int C, int k, int st,
                                                            int Ho, int Wo, long total8, HT* __restrict__ y,
                                                            unsigned char* __restrict__ idx) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int C8 = C / 8;
    const int c8 = (int)(e % C8);
    const long o = e / C8;
    const int j = (int)(o % Wo), i = (int)((o / Wo) % Ho);
    const long b = o / ((long)Wo * Ho);
    float best[8];
    int bi[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -INFINITY;
      bi[q] = 0;
    }
    for (int di = 0; di < k; ++di)
      for (int dj = 0; dj < k; ++dj) {
        const vec_t<HT, 8> v =
            *reinterpret_cast<const vec_t<HT, 8>*>(x + ((b * H + i * st + di) * W + j * st + dj) * C + c8 * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float f = (float)v[q];
          if ((di == 0 && dj == 0) || f > best[q] || f != f) {  // torch: val > maxval || isnan(val): the last NaN wins
            best[q] = f;
            bi[q] = di * k + dj;
          }
        }
      }
    vec_t<HT, 8> out;
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = (HT)best[q];
    *reinterpret_cast<vec_t<HT, 8>*>(y + o * C + c8 * 8) = out;
    if (idx) {
      unsigned long long packed = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) packed |= (unsigned long long)bi[q] << (8 * q);
      *reinterpret_cast<unsigned long long*>(idx + o * C + c8 * 8) = packed;
    }
  }
}

// gather form of the overlapping-window backward: input (i, j) collects dy of every window (oi, oj) that covers it
// and whose argmax is it; times the ReLU mask of the (post-ReLU) pool input
template <typename HT>
__global__ __launch_bounds__(256) void maxpool_k_bwd_kernel(const HT* __restrict__ dy, const unsigned char* __restrict__ idx,
                                                            const HT* __restrict__ post_in, int H, int W, int C, int k,
                                                            int st, int Ho, int Wo, long total8, HT* __restrict__ dx) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total8; e += (long)gridDim.x * blockDim.x) {
    const int C8 = C / 8;
    const int c8 = (int)(e % C8);
    const long pix = e / C8;
    const int j = (int)(pix % W), i = (int)((pix / W) % H);
    const long b = pix / ((long)W * H);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    const int oi0 = i - k + 1 > 0 ? (i - k + 1 + st - 1) / st : 0, oi1 = min(i / st, Ho - 1);
    const int oj0 = j - k + 1 > 0 ? (j - k + 1 + st - 1) / st : 0, oj1 = min(j / st, Wo - 1);
    for (int oi = oi0; oi <= oi1; ++oi)
      for (int oj = oj0; oj <= oj1; ++oj) {
        const long o = ((b * Ho + oi) * Wo + oj) * C + c8 * 8;
        const int pos = (i - oi * st) * k + (j - oj * st);
        const vec_t<HT, 8> g = *reinterpret_cast<const vec_t<HT, 8>*>(dy + o);
        const unsigned long long packed = *reinterpret_cast<const unsigned long long*>(idx + o);
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if ((int)((packed >> (8 * q)) & 0xff) == pos) acc[q] += (float)g[q];
      }
    const vec_t<HT, 8> pin = *reinterpret_cast<const vec_t<HT, 8>*>(post_in + pix * C + c8 * 8);
    vec_t<HT, 8> out;
#pragma unroll
    for (int q = 0; q < 8; ++q) out[q] = (HT)(!((float)pin[q] <= 0.f) ? acc[q] : 0.f);  // relu bwd: NaN passes
    *reinterpret_cast<vec_t<HT, 8>*>(dx + pix * C + c8 * 8) = out;
  }
}

// LPIPS alex conv0 (11x11 / 4, pad 2) input gradient: a thread per input pixel gathers the <= 3 x 3 output taps of its
// stride phase; the 3 image channels accumulate in fp32 (channels 3..7 of the padded input get zero)
template <typename HT>
__global__ __launch_bounds__(256) void alex_conv0_dgrad_kernel(const HT* __restrict__ dpre, const float* __restrict__ w,
                                                               int H, int W, int Ho, int Wo, int Cout, long npix,
                                                               float* __restrict__ d8) {
  constexpr int K = 11, ST = 4, PAD = 2;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const int j = (int)(p % W), i = (int)((p / W) % H);
    const long b = p / ((long)W * H);
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int ki = (i + PAD) % ST; ki < K; ki += ST) {
      const int oi = (i + PAD - ki) / ST;
      if (oi < 0 || oi >= Ho) continue;
      for (int kj = (j + PAD) % ST; kj < K; kj += ST) {
        const int oj = (j + PAD - kj) / ST;
        if (oj < 0 || oj >= Wo) continue;
        const HT* g = dpre + ((b * Ho + oi) * Wo + oj) * Cout;
        const float* wt = w + (ki * K + kj) * 8;
        for (int n = 0; n < Cout; n += 8) {
          const vec_t<HT, 8> gv = *reinterpret_cast<const vec_t<HT, 8>*>(g + n);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float gq = (float)gv[q];
            const float* wq = wt + (long)(n + q) * K * K * 8;
            a0 = fmaf(gq, wq[0], a0);
            a1 = fmaf(gq, wq[1], a1);
            a2 = fmaf(gq, wq[2], a2);
          }
        }
      }
    }
    float4* o = reinterpret_cast<float4*>(d8 + p * 8);
    o[0] = make_float4(a0, a1, a2, 0.f);
    o[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

inline int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

int nbp_vgg_prep(const float* x, int B, int H, int W, int clamp, float m0, float m1, float m2, float s0, float s1,
                 float s2, void* y, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && y && B > 0 && H > 0 && W > 0, "nbp_vgg_prep: bad args");
  const long HW = (long)H * W, n = B * HW;
  NBP_DISPATCH_ALL(dtype, HT, vgg_prep_kernel<HT><<<grid_for(n), 256, 0, S(s)>>>(x, HW, n, clamp, m0, m1, m2, s0, s1, s2,
                                                                              reinterpret_cast<HT*>(y)));
  return check_launch("vgg_prep");
}

int nbp_maxpool2_fwd(const void* x, int B, int H, int W, int C, void* y, unsigned char* idx, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && y && idx && B > 0 && H >= 2 && W >= 2 && C % 8 == 0, "nbp_maxpool2_fwd: bad args");
  const long total8 = (long)B * (H / 2) * (W / 2) * (C / 8);
  NBP_DISPATCH_ALL(dtype, HT, maxpool_fwd_kernel<HT><<<grid_for(total8), 256, 0, S(s)>>>(
      reinterpret_cast<const HT*>(x), H, W, C, total8, reinterpret_cast<HT*>(y), idx));
  return check_launch("maxpool2_fwd");
}

int nbp_maxpool2_bwd(const void* dy, const unsigned char* idx, const void* post_in, int B, int H, int W, int C, void* dx,
                     int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dy && idx && post_in && dx && B > 0 && H >= 2 && W >= 2 && C % 8 == 0, "nbp_maxpool2_bwd: bad args");
  const long total8 = (long)B * H * W * (C / 8);
  NBP_DISPATCH_ALL(dtype, HT, maxpool_bwd_kernel<HT><<<grid_for(total8), 256, 0, S(s)>>>(
      reinterpret_cast<const HT*>(dy), idx, reinterpret_cast<const HT*>(post_in), H, W, C, total8,
      reinterpret_cast<HT*>(dx)));
  return check_launch("maxpool2_bwd");
}

int nbp_maxpool_k_fwd(const void* x, int B, int H, int W, int C, int k, int stride, void* y, unsigned char* idx,
                      int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && y && B > 0 && k > 0 && k * k <= 256 && stride > 0 && H >= k && W >= k && C % 8 == 0,
              "nbp_maxpool_k_fwd: bad args");
  const int Ho = (H - k) / stride + 1, Wo = (W - k) / stride + 1;
  const long total8 = (long)B * Ho * Wo * (C / 8);
  NBP_DISPATCH_ALL(dtype, HT, maxpool_k_fwd_kernel<HT><<<grid_for(total8), 256, 0, S(s)>>>(
      reinterpret_cast<const HT*>(x), H, W, C, k, stride, Ho, Wo, total8, reinterpret_cast<HT*>(y), idx));
  return check_launch("maxpool_k_fwd");
}

int nbp_maxpool_k_bwd(const void* dy, const unsigned char* idx, const void* post_in, int B, int H, int W, int C, int k,
                      int stride, void* dx, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dy && idx && post_in && dx && B > 0 && k > 0 && stride > 0 && H >= k && W >= k && C % 8 == 0,
              "nbp_maxpool_k_bwd: bad args");
  const int Ho = (H - k) / stride + 1, Wo = (W - k) / stride + 1;
  const long total8 = (long)B * H * W * (C / 8);
  NBP_DISPATCH_ALL(dtype, HT, maxpool_k_bwd_kernel<HT><<<grid_for(total8), 256, 0, S(s)>>>(
      reinterpret_cast<const HT*>(dy), idx, reinterpret_cast<const HT*>(post_in), H, W, C, k, stride, Ho, Wo, total8,
      reinterpret_cast<HT*>(dx)));
  return check_launch("maxpool_k_bwd");
}

int nbp_alex_conv0_input_grad(const void* dpre, const float* w, int B, int H, int W, int Ho, int Wo, int Cout,
                              float* d8, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dpre && w && d8 && B > 0 && H > 0 && W > 0 && Cout % 8 == 0, "nbp_alex_conv0_input_grad: bad args");
  NBP_REQUIRE(Ho == (H + 4 - 11) / 4 + 1 && Wo == (W + 4 - 11) / 4 + 1, "nbp_alex_conv0_input_grad: output geometry");
  const long npix = (long)B * H * W;
  NBP_DISPATCH_ALL(dtype, HT, alex_conv0_dgrad_kernel<HT><<<grid_for(npix), 256, 0, S(s)>>>(
      reinterpret_cast<const HT*>(dpre), w, H, W, Ho, Wo, Cout, npix, d8));
  return check_launch("alex_conv0_input_grad");
}

size_t nbp_feat_dist_workspace_doubles(long n) {
  long g = (n + 255) / 256;
  return (size_t)(g > 2048 ? 2048 : (g < 1 ? 1 : g));
}

int nbp_feat_dist_fwd(const void* a, const void* b, long n, int mode, double scale, double* ws, float* out,
                      int dtype, nbp_stream_t s) {
  NBP_REQUIRE(a && b && ws && out && n > 0 && (mode == 0 || mode == 1), "nbp_feat_dist_fwd: bad args");
  const int g = (int)nbp_feat_dist_workspace_doubles(n);
  NBP_DISPATCH_ALL(dtype, HT, feat_dist_fwd<HT><<<g, 256, 0, S(s)>>>(reinterpret_cast<const HT*>(a),
                                                                     reinterpret_cast<const HT*>(b), n, mode, ws));
  feat_dist_finalize<<<1, 64, 0, S(s)>>>(ws, g, scale, out);
  return check_launch("feat_dist_fwd");
}

int nbp_feat_dist_bwd(const void* a, const void* b, long n, int mode, float scale, int relu_mask, const float* up,
                      void* da, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(a && b && up && da && n > 0 && (mode == 0 || mode == 1), "nbp_feat_dist_bwd: bad args");
  NBP_DISPATCH_ALL(dtype, HT, feat_dist_bwd<HT><<<grid_for(n), 256, 0, S(s)>>>(
      reinterpret_cast<const HT*>(a), reinterpret_cast<const HT*>(b), n, mode, scale, relu_mask, up,
      reinterpret_cast<HT*>(da)));
  return check_launch("feat_dist_bwd");
}

int nbp_vgg_input_grad(const float* d8, const float* x, int B, int H, int W, int clamp, float s0, float s1, float s2,
                       float* dx, nbp_stream_t s) {
  NBP_REQUIRE(d8 && x && dx && B > 0 && H > 0 && W > 0, "nbp_vgg_input_grad: bad args");
  const long HW = (long)H * W, n = B * HW;
  vgg_input_grad_kernel<<<grid_for(n), 256, 0, S(s)>>>(d8, x, HW, n, clamp, s0, s1, s2, dx);
  return check_launch("vgg_input_grad");
}

int nbp_add_relu_masked(void* d, const void* g, const void* post, long n, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(d && g && post && n > 0, "nbp_add_relu_masked: bad args");
  NBP_DISPATCH_ALL(dtype, HT, add_relu_masked_kernel<HT><<<grid_for(n), 256, 0, S(s)>>>(
      reinterpret_cast<HT*>(d), reinterpret_cast<const HT*>(g), reinterpret_cast<const HT*>(post), n));
  return check_launch("add_relu_masked");
}

// lanes per pixel group: the power of two >= the 16-byte chunk count, at most 64 (then V = ceil(chunks / 64) <= 4)
inline int tap_lanes(int nch) {
  int G = 1;
  while (G < nch && G < 64) G <<= 1;
  return G;
}
#define NBP_TAP_DISPATCH(KERNEL, GRID, ...)                                                   \
  switch (C / 8 <= 64 ? tap_lanes(C / 8) : (C / 8 <= 128 ? 128 : 256)) {                    \
    case 1: KERNEL<1, 1, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                   \
    case 2: KERNEL<2, 1, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                   \
    case 4: KERNEL<4, 1, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                   \
    case 8: KERNEL<8, 1, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                   \
    case 16: KERNEL<16, 1, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                 \
    case 32: KERNEL<32, 1, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                 \
    case 64: KERNEL<64, 1, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                 \
    case 128: KERNEL<64, 2, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                \
    default: KERNEL<64, 4, HT><<<GRID, 256, 0, S(s)>>>(__VA_ARGS__); break;                 \
  }

inline int lpips_chunks(long HW, int N) {
  long c = (HW + 2047) / 2048, want = (1024 + N - 1) / N;
  if (c > want) c = want;
  return (int)(c < 1 ? 1 : (c > 1024 ? 1024 : c));
}

size_t nbp_lpips_tap_workspace_doubles(int N, long HW) { return (size_t)N * lpips_chunks(HW, N); }

int nbp_lpips_tap_fwd(const void* a, const void* b, const float* w, int N, long HW, int C, int accumulate, double* ws,
                      float* out, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(a && b && w && ws && out && N > 0 && N <= 65535 && HW > 0 && C % 8 == 0 && C <= 2048,
              "nbp_lpips_tap_fwd: bad args");
  const int chunks = lpips_chunks(HW, N);
  NBP_DISPATCH_ALL(dtype, HT, {
    const HT* pa = reinterpret_cast<const HT*>(a);
    const HT* pb = reinterpret_cast<const HT*>(b);
    const dim3 g(chunks, N);
    NBP_TAP_DISPATCH(lpips_tap_fwd, g, pa, pb, w, HW, C, chunks, ws);
  });
  lpips_finalize<<<cdiv(N, 256), 256, 0, S(s)>>>(ws, N, chunks, 1.0 / (double)HW, accumulate, out);
  return check_launch("lpips_tap_fwd");
}

int nbp_lpips_tap_bwd(const void* a, const void* b, const float* w, int N, long HW, int C, const float* up, void* da,
                      int dtype, nbp_stream_t s) {
  NBP_REQUIRE(a && b && w && up && da && N > 0 && HW > 0 && C % 8 == 0 && C <= 2048, "nbp_lpips_tap_bwd: bad args");
  const long npix = (long)N * HW;
  NBP_DISPATCH_ALL(dtype, HT, {
    const HT* pa = reinterpret_cast<const HT*>(a);
    const HT* pb = reinterpret_cast<const HT*>(b);
    const long gpb = 256 / tap_lanes(C / 8);
    long g = (npix + gpb - 1) / gpb;
    if (g > 8192) g = 8192;
    NBP_TAP_DISPATCH(lpips_tap_bwd, (unsigned)g, pa, pb, w, HW, C, npix, up, reinterpret_cast<HT*>(da));
  });
  return check_launch("lpips_tap_bwd");
}

}  // extern "C"
