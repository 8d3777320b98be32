// Physics branch: crosstalk PSF (NewBP_model/newbp_layer.py:88-173), exposure alignment and the
// physics-consistency losses (NewBP_model/losses.py:158-220) and metric (metrics/phys_consistency.py:193-368).
// Layout: NCHW fp32 (the reference's public layout; these tensors are 3-channel images).
#include <math.h>
#include <string.h>

#include "nbp_common.h"

using namespace nbp;

namespace {

constexpr int kBlk = 256;

__device__ __forceinline__ int reflect_idx(int i, int n) {  // F.pad(mode='reflect'), pad < n
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}
__device__ __forceinline__ int clampi(int i, int lo, int hi) { return i < lo ? lo : (i > hi ? hi : i); }
__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }
__device__ __forceinline__ float fsign(float v) { return v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f); }

// outputs q in [lo, hi] with clamp(q + d, 0, n-1) == p (empty when lo > hi)
__device__ __forceinline__ void rep_range(int p, int d, int n, int& lo, int& hi) {
  if (n == 1) { lo = 0; hi = 0; return; }
  if (p == 0) { lo = 0; hi = min(-d, n - 1); return; }
  if (p == n - 1) { lo = max(n - 1 - d, 0); hi = n - 1; return; }
  lo = hi = p - d;
  if (lo < 0 || lo >= n) { lo = 1; hi = 0; }
}

// ---------------------------------------------------------------- depthwise KxK conv (NCHW)
// pad: 0 zeros, 1 replicate, 2 reflect.  k: [C][KH*KW] or [1][KH*KW] when k_shared.
template <int PAD>
__global__ void dw_conv_fwd(const float* __restrict__ x, const float* __restrict__ k, int k_shared, float* __restrict__ y,
                            int N, int C, int H, int W, int KH, int KW, int pre_clamp) {
  const int total = N * C * H * W;  // < 2^31 (host check): 32-bit index arithmetic
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W, h = hw % H;
    const int plane = hw / H;
    const int c = plane % C;
    const float* xp = x + (long)plane * H * W;
    const float* kc = k + (k_shared ? 0 : (long)c * KH * KW);
    float acc = 0.f;
    for (int a = 0; a < KH; ++a) {
      int hh = h + a - KH / 2;
      for (int b = 0; b < KW; ++b) {
        int ww = w + b - KW / 2;
        float v;
        if (PAD == 0) {
          v = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? xp[(long)hh * W + ww] : 0.f;
        } else if (PAD == 1) {
          v = xp[(long)clampi(hh, 0, H - 1) * W + clampi(ww, 0, W - 1)];
        } else {
          v = xp[(long)reflect_idx(hh, H) * W + reflect_idx(ww, W)];
        }
        if (pre_clamp) v = clamp01(v);
        acc = fmaf(kc[a * KW + b], v, acc);
      }
    }
    y[i] = acc;
  }
}

// adjoint of the zero-padded depthwise conv: gx(p) = sum_t k[t] * gy(p - (t - K/2))
__global__ void dw_conv_bwd_zero(const float* __restrict__ gy, const float* __restrict__ k, int k_shared,
                                 float* __restrict__ gx, int N, int C, int H, int W, int KH, int KW) {
  const int total = N * C * H * W;  // < 2^31 (host check): 32-bit index arithmetic
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W, h = hw % H;
    const int plane = hw / H;
    const int c = plane % C;
    const float* gp = gy + (long)plane * H * W;
    const float* kc = k + (k_shared ? 0 : (long)c * KH * KW);
    float acc = 0.f;
    for (int a = 0; a < KH; ++a) {
      int hh = h - (a - KH / 2);
      if (hh < 0 || hh >= H) continue;
      for (int b = 0; b < KW; ++b) {
        int ww = w - (b - KW / 2);
        if (ww < 0 || ww >= W) continue;
        acc = fmaf(kc[a * KW + b], gp[(long)hh * W + ww], acc);
      }
    }
    gx[i] = acc;
  }
}

// ---------------------------------------------------------------- fused physics L1 (sRGB / raw training losses)
// d = PSF_pad(pre?(bhat)) - clamp?(pre?(a) * ratio) ; partial sums of |d| per block ; sign(d) map.
// ratio: [N*C] per (sample, channel) when ratio_full == 0, else a full [N,C,H,W] map.
template <int PAD>
__global__ void phys_l1_fwd(const float* __restrict__ bhat, const float* __restrict__ a, const float* __restrict__ ratio,
                            int ratio_full, const float* __restrict__ k, int k_shared, int N, int C, int H, int W, int KH,
                            int KW, int clamp_bhat, int clamp_a_in, int clamp_align, double* __restrict__ partial,
                            float* __restrict__ sign_map) {
  __shared__ double red[16];
  const int total = N * C * H * W;  // < 2^31 (host check): 32-bit index arithmetic
  double s = 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W, h = hw % H;
    const int plane = hw / H;
    const int c = plane % C;
    const float* xp = bhat + (long)plane * H * W;
    const float* kc = k + (k_shared ? 0 : (long)c * KH * KW);
    float y = 0.f;
    for (int aa = 0; aa < KH; ++aa) {
      int hh = h + aa - KH / 2;
      for (int bb = 0; bb < KW; ++bb) {
        int ww = w + bb - KW / 2;
        float v;
        if (PAD == 0) {
          v = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? xp[(long)hh * W + ww] : 0.f;
          if (clamp_bhat) v = clamp01(v);
        } else {
          v = xp[(long)clampi(hh, 0, H - 1) * W + clampi(ww, 0, W - 1)];
          if (clamp_bhat) v = clamp01(v);
        }
        y = fmaf(kc[aa * KW + bb], v, y);
      }
    }
    float av = a[i];
    if (clamp_a_in) av = clamp01(av);
    const float r = ratio_full ? ratio[i] : ratio[plane];
    float al = av * r;
    if (clamp_align) al = clamp01(al);
    const float d = y - al;
    s += fabsf(d);
    if (sign_map) sign_map[i] = fsign(d);
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// grad wrt bhat: up[0] * scale * mask(bhat) * PSF^T(sign) ; PAD 0: zero-pad adjoint, 1: replicate adjoint
template <int PAD>
__global__ void phys_l1_bwd(const float* __restrict__ sign_map, const float* __restrict__ bhat,
                            const float* __restrict__ k, int k_shared, const float* __restrict__ up, float scale,
                            int N, int C, int H, int W, int KH, int KW, int clamp_bhat, float* __restrict__ gx) {
  const int total = N * C * H * W;  // < 2^31 (host check): 32-bit index arithmetic
  const float g0 = up[0] * scale;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W, h = hw % H;
    const int plane = hw / H;
    const int c = plane % C;
    const float* sp = sign_map + (long)plane * H * W;
    const float* kc = k + (k_shared ? 0 : (long)c * KH * KW);
    float acc = 0.f;
    if (PAD == 0) {
      for (int aa = 0; aa < KH; ++aa) {
        int hh = h - (aa - KH / 2);
        if (hh < 0 || hh >= H) continue;
        for (int bb = 0; bb < KW; ++bb) {
          int ww = w - (bb - KW / 2);
          if (ww < 0 || ww >= W) continue;
          acc = fmaf(kc[aa * KW + bb], sp[(long)hh * W + ww], acc);
        }
      }
    } else {
      // replicate pad: output q reads clamp(q + off); the adjoint gathers every (q, off) landing on p
      for (int aa = 0; aa < KH; ++aa) {
        int qh0, qh1;
        rep_range(h, aa - KH / 2, H, qh0, qh1);
        for (int bb = 0; bb < KW; ++bb) {
          int qw0, qw1;
          rep_range(w, bb - KW / 2, W, qw0, qw1);
          const float kv = kc[aa * KW + bb];
          for (int qh = qh0; qh <= qh1; ++qh)
            for (int qw = qw0; qw <= qw1; ++qw) acc = fmaf(kv, sp[(long)qh * W + qw], acc);
        }
      }
    }
    float m = 1.f;
    if (clamp_bhat) {
      const float b = bhat[i];
      m = (b >= 0.f && b <= 1.f) ? 1.f : 0.f;
    }
    gx[i] = g0 * acc * m;
  }
}

// ---------------------------------------------------------------- raw physics L1, groups = 1 (full / expanded PSF)
// PhysicsConsistencyLoss's groups == 1 branch (NewBP_model/losses.py:182-191): a [Co][C][KH][KW] kernel (the caller
// expands a [Co][1] one along C) over the replicate-padded prediction,
//   yhat[n][co][h][w] = sum_{c,a,b} k[co][c][a][b] * bhat[n][c][clamp(h + a - KH/2)][clamp(w + b - KW/2)],
// compared with al = clamp?(a * ratio) under torch's channel broadcast of F.l1_loss: Cb = max(Co, Ca) output
// channels, yhat's channel min(cb, Co - 1) (Co == 1 broadcasts), al's min(cb, Ca - 1).  Partial sums of |d| per
// block, sign(d) map [N][Cb][H][W].
__global__ void phys_full_fwd(const float* __restrict__ bhat, const float* __restrict__ a, const float* __restrict__ ratio,
                              int ratio_full, const float* __restrict__ k, int N, int C, int Co, int Ca, int H, int W,
                              int KH, int KW, int clamp_align, double* __restrict__ partial,
                              float* __restrict__ sign_map) {
  __shared__ double red[16];
  const int Cb = Co > Ca ? Co : Ca;
  const int total = N * Cb * H * W;  // < 2^31 (host check)
  double s = 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W, h = hw % H;
    const int plane = hw / H;
    const int cb = plane % Cb, n = plane / Cb;
    const int co = Co == 1 ? 0 : cb, ca = Ca == 1 ? 0 : cb;
    float y = 0.f;
    for (int c = 0; c < C; ++c) {
      const float* xp = bhat + ((long)n * C + c) * H * W;
      const float* kc = k + ((long)co * C + c) * KH * KW;
      for (int aa = 0; aa < KH; ++aa) {
        const int hh = clampi(h + aa - KH / 2, 0, H - 1);
        for (int bb = 0; bb < KW; ++bb)
          y = fmaf(kc[aa * KW + bb], xp[(long)hh * W + clampi(w + bb - KW / 2, 0, W - 1)], y);
      }
    }
    const long ai = (((long)n * Ca + ca) * H + h) * W + w;
    const float r = ratio_full ? ratio[ai] : ratio[n * Ca + ca];
    float al = a[ai] * r;
    if (clamp_align) al = clamp01(al);
    const float d = y - al;
    s += fabsf(d);
    if (sign_map) sign_map[i] = fsign(d);
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// gx[n][c][p] = up[0] * scale * sum_cb sum_{a,b} k[co(cb)][c][a][b] * sum_{q: clamp(q + off) == p} sign[n][cb][q]
__global__ void phys_full_bwd(const float* __restrict__ sign_map, const float* __restrict__ k, const float* __restrict__ up,
                              float scale, int N, int C, int Co, int Cb, int H, int W, int KH, int KW,
                              float* __restrict__ gx) {
  const int total = N * C * H * W;
  const float g0 = up[0] * scale;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W, h = hw % H;
    const int plane = hw / H;
    const int c = plane % C, n = plane / C;
    float acc = 0.f;
    for (int cb = 0; cb < Cb; ++cb) {
      const float* sp = sign_map + ((long)n * Cb + cb) * H * W;
      const float* kc = k + ((long)(Co == 1 ? 0 : cb) * C + c) * KH * KW;
      for (int aa = 0; aa < KH; ++aa) {
        int qh0, qh1;
        rep_range(h, aa - KH / 2, H, qh0, qh1);
        for (int bb = 0; bb < KW; ++bb) {
          int qw0, qw1;
          rep_range(w, bb - KW / 2, W, qw0, qw1);
          const float kv = kc[aa * KW + bb];
          for (int qh = qh0; qh <= qh1; ++qh)
            for (int qw = qw0; qw <= qw1; ++qw) acc = fmaf(kv, sp[(long)qh * W + qw], acc);
        }
      }
    }
    gx[i] = g0 * acc;
  }
}

// grad wrt the short exposure A (the reference's losses are plain autograd, NewBP_model/losses.py:158-220):
// al = clamp?(pre?(a) * r) enters d = yhat - al with a minus sign, so
//   ga[n][ca][p] = -up[0] * scale * sum_{cb -> ca} sign[n][cb][p] * r * mask_align * mask_a
// (torch's clamp backward passes the gradient where lo <= x <= hi; cb -> ca: F.l1_loss's channel broadcast, every cb
// when Ca == 1, else cb == ca).  Depthwise losses: Cb = Ca = C.
__global__ void phys_a_bwd(const float* __restrict__ sign_map, const float* __restrict__ a, const float* __restrict__ ratio,
                           int ratio_full, int N, int Ca, int Cb, int H, int W, int clamp_a_in, int clamp_align,
                           const float* __restrict__ up, float scale, float* __restrict__ ga) {
  const int total = N * Ca * H * W;
  const float g0 = -up[0] * scale;
  const int HW = H * W;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int p = i % HW, plane = i / HW;
    const int ca = plane % Ca, n = plane / Ca;
    const float a0 = a[i];
    const float av = clamp_a_in ? clamp01(a0) : a0;
    const float r = ratio_full ? ratio[i] : ratio[plane];
    const float al = av * r;
    float m = (!clamp_align || (al >= 0.f && al <= 1.f)) ? r : 0.f;
    if (clamp_a_in && !(a0 >= 0.f && a0 <= 1.f)) m = 0.f;
    float acc = 0.f;
    if (Ca == Cb) acc = sign_map[i];
    else
      for (int cb = 0; cb < Cb; ++cb) acc += sign_map[((long)n * Cb + cb) * HW + p];
    ga[i] = g0 * acc * m;
  }
}

// fixed-order sum of block partials -> out[0] = scale * sum
__global__ void finalize_sum(const double* __restrict__ partial, int n, double scale, float* __restrict__ out) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) out[0] = (float)(s * scale);
}

// ---------------------------------------------------------------- phys_cons metric core (full [Co,Ci,kh,kw] PSF)
// one block row per sample n (grid.y); output pixels of the (possibly cropped) region.
template <int PAD>
__global__ void phys_cons_core(const float* __restrict__ pred, const float* __restrict__ obs,
                               const float* __restrict__ psf, const float* __restrict__ ratio, int ratio_mode,
                               int N, int Ci, int Co, int H, int W, int KH, int KW, int crop_valid, int clamp01_out,
                               int charbonnier, float eps, float* __restrict__ amap, double* __restrict__ partial) {
  __shared__ double red[16];
  const int n = blockIdx.y;
  const int ph = crop_valid ? KH / 2 : 0, pw = crop_valid ? KW / 2 : 0;
  const int Ho = H - 2 * ph, Wo = W - 2 * pw;
  const long per = (long)Ho * Wo;
  double s = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < per; i += (long)gridDim.x * blockDim.x) {
    const int wo = i % Wo, ho = i / Wo;
    const int h = ho + ph, w = wo + pw;
    for (int co = 0; co < Co; ++co) {
      float y = 0.f;
      for (int ci = 0; ci < Ci; ++ci) {
        const float* xp = pred + ((long)n * Ci + ci) * H * W;
        const float* kp = psf + ((long)co * Ci + ci) * KH * KW;
        for (int a = 0; a < KH; ++a) {
          int hh = h + a - KH / 2;
          for (int b = 0; b < KW; ++b) {
            int ww = w + b - KW / 2;
            float v;
            if (PAD == 0) {
              v = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? xp[(long)hh * W + ww] : 0.f;
            } else if (PAD == 1) {
              v = xp[(long)clampi(hh, 0, H - 1) * W + clampi(ww, 0, W - 1)];
            } else {
              v = xp[(long)reflect_idx(hh, H) * W + reflect_idx(ww, W)];
            }
            y = fmaf(kp[a * KW + b], v, y);
          }
        }
      }
      // ratio_mode: 0 per-sample [N], 1 [N,1,H,W], 2 [N,Co,H,W]
      float r;
      if (ratio_mode == 0) r = ratio[n];
      else if (ratio_mode == 1) r = ratio[(long)n * H * W + (long)h * W + w];
      else r = ratio[((long)n * Co + co) * H * W + (long)h * W + w];
      y = y * r;
      if (clamp01_out) y = clamp01(y);
      const float d = y - obs[((long)n * Co + co) * H * W + (long)h * W + w];
      const float ad = fabsf(d);
      s += charbonnier ? (double)sqrtf(d * d + eps * eps) : (double)ad;
      if (amap) amap[((long)n * Co + co) * per + i] = ad;
    }
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) partial[(long)n * gridDim.x + blockIdx.x] = s;
}

// per-sample means and the batch reduction: out[0..N-1] per-sample, out[N] = mean, out[N+1] = sum
__global__ void phys_cons_finalize(const double* __restrict__ partial, int nblk, int N, double inv_count,
                                   float* __restrict__ out) {
  __shared__ float vals[1024];
  for (int n = threadIdx.x; n < N; n += blockDim.x) {
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += partial[(long)n * nblk + b];
    out[n] = (float)(s * inv_count);
    if (n < 1024) vals[n] = out[n];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sm = 0.f;  // torch reduces the [N] fp32 vector; N is small, order n=0..N-1
    for (int n = 0; n < N; ++n) sm += out[n];
    out[N] = sm / (float)N;
    out[N + 1] = sm;
  }
}

// align_exposure_srgb (losses.py:195-203): out = clamp(a * ratio, 0, 1)
__global__ void align_kernel(const float* __restrict__ a, const float* __restrict__ ratio, int ratio_full,
                             float* __restrict__ out, long total, long HW) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const float r = ratio_full ? ratio[i] : ratio[i / HW];
    out[i] = clamp01(a[i] * r);
  }
}

__global__ void all_finite_kernel(const float* __restrict__ x, long n, int* __restrict__ flag) {
  int bad = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

inline int grid_for(long total) {
  long g = (total + kBlk - 1) / kBlk;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" {

int nbp_psf_normalize_host(const float* k, int n_kernels, int len, float* out) {
  NBP_REQUIRE(k && out && n_kernels > 0 && len > 0, "nbp_psf_normalize_host: bad arguments");
  for (int i = 0; i < n_kernels; ++i) {
    // torch (AVX512 CPU) sums a row of <= 16 floats with 8 interleaved accumulators combined in order.
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < len; ++j) acc[j % 8] += k[(long)i * len + j];
    float s = 0.f;
    for (int j = 0; j < 8; ++j) s += acc[j];
    if (s < 1e-12f) s = 1e-12f;  // clamp_min(1e-12) (newbp_layer.py:105)
    for (int j = 0; j < len; ++j) out[(long)i * len + j] = k[(long)i * len + j] / s;
  }
  return NBP_OK;
}

int nbp_dwconv_nchw_fwd(const float* x, const float* k, int k_shared, float* y, int N, int C, int H, int W, int KH,
                        int KW, int pad_mode, int pre_clamp, nbp_stream_t s) {
  NBP_REQUIRE(x && k && y && N > 0 && C > 0 && H > 0 && W > 0 && (KH & 1) && (KW & 1), "nbp_dwconv_nchw_fwd: bad args");
  NBP_REQUIRE((long)N * C * H * W < (1L << 31), "physics kernels: N*C*H*W must be < 2^31");
  NBP_REQUIRE(pad_mode >= 0 && pad_mode <= 2, "nbp_dwconv_nchw_fwd: pad_mode");
  NBP_REQUIRE(pad_mode != 2 || (KH / 2 < H && KW / 2 < W), "reflect padding needs pad < size");
  const long total = (long)N * C * H * W;
  if (pad_mode == 0) dw_conv_fwd<0><<<grid_for(total), kBlk, 0, S(s)>>>(x, k, k_shared, y, N, C, H, W, KH, KW, pre_clamp);
  else if (pad_mode == 1) dw_conv_fwd<1><<<grid_for(total), kBlk, 0, S(s)>>>(x, k, k_shared, y, N, C, H, W, KH, KW, pre_clamp);
  else dw_conv_fwd<2><<<grid_for(total), kBlk, 0, S(s)>>>(x, k, k_shared, y, N, C, H, W, KH, KW, pre_clamp);
  return check_launch("dw_conv_fwd");
}

int nbp_dwconv_nchw_bwd_zero(const float* gy, const float* k, int k_shared, float* gx, int N, int C, int H, int W,
                             int KH, int KW, nbp_stream_t s) {
  NBP_REQUIRE(gy && k && gx && N > 0 && C > 0 && H > 0 && W > 0 && (KH & 1) && (KW & 1), "nbp_dwconv_nchw_bwd_zero: bad args");
  NBP_REQUIRE((long)N * C * H * W < (1L << 31), "physics kernels: N*C*H*W must be < 2^31");
  const long total = (long)N * C * H * W;
  dw_conv_bwd_zero<<<grid_for(total), kBlk, 0, S(s)>>>(gy, k, k_shared, gx, N, C, H, W, KH, KW);
  return check_launch("dw_conv_bwd_zero");
}

size_t nbp_phys_l1_workspace_doubles(int N, int C, int H, int W) {
  return (size_t)grid_for((long)N * C * H * W);
}

int nbp_phys_l1_fwd(const float* bhat, const float* a, const float* ratio, int ratio_full, const float* k, int k_shared,
                    int N, int C, int H, int W, int KH, int KW, int pad_mode, int clamp_bhat, int clamp_a_in,
                    int clamp_align, double* ws, float* loss, float* sign_map, nbp_stream_t s) {
  NBP_REQUIRE(bhat && a && ratio && k && ws && loss && N > 0 && C > 0 && H > 0 && W > 0, "nbp_phys_l1_fwd: bad args");
  NBP_REQUIRE((KH & 1) && (KW & 1) && (pad_mode == 0 || pad_mode == 1), "nbp_phys_l1_fwd: kernel/pad");
  NBP_REQUIRE((long)N * C * H * W < (1L << 31), "physics kernels: N*C*H*W must be < 2^31");
  const long total = (long)N * C * H * W;
  const int g = grid_for(total);
  if (pad_mode == 0)
    phys_l1_fwd<0><<<g, kBlk, 0, S(s)>>>(bhat, a, ratio, ratio_full, k, k_shared, N, C, H, W, KH, KW, clamp_bhat,
                                          clamp_a_in, clamp_align, ws, sign_map);
  else
    phys_l1_fwd<1><<<g, kBlk, 0, S(s)>>>(bhat, a, ratio, ratio_full, k, k_shared, N, C, H, W, KH, KW, clamp_bhat,
                                          clamp_a_in, clamp_align, ws, sign_map);
  finalize_sum<<<1, 256, 0, S(s)>>>(ws, g, 1.0 / (double)total, loss);
  return check_launch("phys_l1_fwd");
}

int nbp_phys_l1_bwd(const float* sign_map, const float* bhat, const float* k, int k_shared, const float* up, int N,
                    int C, int H, int W, int KH, int KW, int pad_mode, int clamp_bhat, float* gx, nbp_stream_t s) {
  NBP_REQUIRE(sign_map && k && up && gx && (!clamp_bhat || bhat), "nbp_phys_l1_bwd: bad args");
  NBP_REQUIRE(pad_mode == 0 || pad_mode == 1, "nbp_phys_l1_bwd: pad");
  NBP_REQUIRE((long)N * C * H * W < (1L << 31), "physics kernels: N*C*H*W must be < 2^31");
  const long total = (long)N * C * H * W;
  const float scale = (float)(1.0 / (double)total);
  if (pad_mode == 0)
    phys_l1_bwd<0><<<grid_for(total), kBlk, 0, S(s)>>>(sign_map, bhat, k, k_shared, up, scale, N, C, H, W, KH, KW,
                                                        clamp_bhat, gx);
  else
    phys_l1_bwd<1><<<grid_for(total), kBlk, 0, S(s)>>>(sign_map, bhat, k, k_shared, up, scale, N, C, H, W, KH, KW,
                                                        clamp_bhat, gx);
  return check_launch("phys_l1_bwd");
}

int nbp_phys_full_fwd(const float* bhat, const float* a, const float* ratio, int ratio_full, const float* k, int N,
                      int C, int Co, int Ca, int H, int W, int KH, int KW, int clamp_align, double* ws, float* loss,
                      float* sign_map, nbp_stream_t s) {
  NBP_REQUIRE(bhat && a && ratio && k && ws && loss && N > 0 && C > 0 && Co > 0 && Ca > 0 && H > 0 && W > 0,
              "nbp_phys_full_fwd: bad args");
  NBP_REQUIRE((KH & 1) && (KW & 1), "nbp_phys_full_fwd: odd kernel sizes");
  NBP_REQUIRE(Co == Ca || Co == 1 || Ca == 1, "nbp_phys_full_fwd: channels %d and %d do not broadcast", Co, Ca);
  const int Cb = Co > Ca ? Co : Ca;
  NBP_REQUIRE((long)N * (Cb > C ? Cb : C) * H * W < (1L << 31), "physics kernels: N*C*H*W must be < 2^31");
  const long total = (long)N * Cb * H * W;
  const int g = grid_for(total);
  phys_full_fwd<<<g, kBlk, 0, S(s)>>>(bhat, a, ratio, ratio_full, k, N, C, Co, Ca, H, W, KH, KW, clamp_align, ws,
                                       sign_map);
  finalize_sum<<<1, 256, 0, S(s)>>>(ws, g, 1.0 / (double)total, loss);
  return check_launch("phys_full_fwd");
}

int nbp_phys_full_bwd(const float* sign_map, const float* k, const float* up, int N, int C, int Co, int Ca, int H, int W,
                      int KH, int KW, float* gx, nbp_stream_t s) {
  NBP_REQUIRE(sign_map && k && up && gx && N > 0 && C > 0 && H > 0 && W > 0, "nbp_phys_full_bwd: bad args");
  NBP_REQUIRE(Co == Ca || Co == 1 || Ca == 1, "nbp_phys_full_bwd: channels %d and %d do not broadcast", Co, Ca);
  const int Cb = Co > Ca ? Co : Ca;
  NBP_REQUIRE((long)N * (Cb > C ? Cb : C) * H * W < (1L << 31), "physics kernels: N*C*H*W must be < 2^31");
  const long total = (long)N * C * H * W;
  const float scale = (float)(1.0 / ((double)N * Cb * H * W));
  phys_full_bwd<<<grid_for(total), kBlk, 0, S(s)>>>(sign_map, k, up, scale, N, C, Co, Cb, H, W, KH, KW, gx);
  return check_launch("phys_full_bwd");
}

int nbp_phys_a_bwd(const float* sign_map, const float* a, const float* ratio, int ratio_full, int N, int Ca, int Cb, int H,
                   int W, int clamp_a_in, int clamp_align, const float* up, float* ga, nbp_stream_t s) {
  NBP_REQUIRE(sign_map && a && ratio && up && ga && N > 0 && Ca > 0 && Cb > 0 && H > 0 && W > 0,
              "nbp_phys_a_bwd: bad args");
  NBP_REQUIRE(Ca == Cb || Ca == 1, "nbp_phys_a_bwd: A's %d channels do not broadcast to %d", Ca, Cb);
  NBP_REQUIRE((long)N * Cb * H * W < (1L << 31), "physics kernels: N*C*H*W must be < 2^31");
  const long total = (long)N * Ca * H * W;
  const float scale = (float)(1.0 / ((double)N * Cb * H * W));
  phys_a_bwd<<<grid_for(total), kBlk, 0, S(s)>>>(sign_map, a, ratio, ratio_full, N, Ca, Cb, H, W, clamp_a_in,
                                                 clamp_align, up, scale, ga);
  return check_launch("phys_a_bwd");
}

size_t nbp_phys_cons_workspace_doubles(int N, int H, int W) {
  long per = (long)H * W;
  int g = (int)((per + kBlk - 1) / kBlk);
  if (g > 256) g = 256;
  return (size_t)N * g;
}

int nbp_phys_cons(const float* pred, const float* obs, const float* psf, const float* ratio, int ratio_mode, int N,
                  int Ci, int Co, int H, int W, int KH, int KW, int pad_mode, int crop_valid, int clamp01_out,
                  int charbonnier, float eps, float* amap, double* ws, float* out, nbp_stream_t s) {
  NBP_REQUIRE(pred && obs && psf && ratio && ws && out && N > 0 && Ci > 0 && Co > 0, "nbp_phys_cons: bad args");
  NBP_REQUIRE((KH & 1) && (KW & 1) && pad_mode >= 0 && pad_mode <= 2 && ratio_mode >= 0 && ratio_mode <= 2,
              "nbp_phys_cons: kernel/pad/ratio");
  NBP_REQUIRE(!crop_valid || (H > 2 * (KH / 2) && W > 2 * (KW / 2)), "nbp_phys_cons: crop larger than image");
  NBP_REQUIRE(pad_mode != 2 || (KH / 2 < H && KW / 2 < W), "reflect padding needs pad < size");
  NBP_REQUIRE(N <= 1024, "nbp_phys_cons: N <= 1024");
  const int ph = crop_valid ? KH / 2 : 0, pw = crop_valid ? KW / 2 : 0;
  const long per = (long)(H - 2 * ph) * (W - 2 * pw);
  int g = (int)((per + kBlk - 1) / kBlk);
  if (g > 256) g = 256;
  dim3 grid(g, N);
  if (pad_mode == 0)
    phys_cons_core<0><<<grid, kBlk, 0, S(s)>>>(pred, obs, psf, ratio, ratio_mode, N, Ci, Co, H, W, KH, KW, crop_valid,
                                                clamp01_out, charbonnier, eps, amap, ws);
  else if (pad_mode == 1)
    phys_cons_core<1><<<grid, kBlk, 0, S(s)>>>(pred, obs, psf, ratio, ratio_mode, N, Ci, Co, H, W, KH, KW, crop_valid,
                                                clamp01_out, charbonnier, eps, amap, ws);
  else
    phys_cons_core<2><<<grid, kBlk, 0, S(s)>>>(pred, obs, psf, ratio, ratio_mode, N, Ci, Co, H, W, KH, KW, crop_valid,
                                                clamp01_out, charbonnier, eps, amap, ws);
  phys_cons_finalize<<<1, 256, 0, S(s)>>>(ws, g, N, 1.0 / (double)(per * Co), out);
  return check_launch("phys_cons");
}

int nbp_align_exposure(const float* a, const float* ratio, int ratio_full, float* out, int N, int C, long HW,
                       nbp_stream_t s) {
  NBP_REQUIRE(a && ratio && out && N > 0 && C > 0 && HW > 0, "nbp_align_exposure: bad args");
  const long total = (long)N * C * HW;
  align_kernel<<<grid_for(total), kBlk, 0, S(s)>>>(a, ratio, ratio_full, out, total, HW);
  return check_launch("align_exposure");
}

int nbp_all_finite(const float* x, long n, int* flag_dev, nbp_stream_t s) {
  NBP_REQUIRE(x && flag_dev && n >= 0, "nbp_all_finite: bad args");
  hipMemsetAsync(flag_dev, 0, sizeof(int), S(s));
  if (n > 0) all_finite_kernel<<<grid_for(n), kBlk, 0, S(s)>>>(x, n, flag_dev);
  return check_launch("all_finite");
}

}  // extern "C"
