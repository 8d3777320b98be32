// Validation metrics on device:
//   * PSNR per sample with float64 error sums: psnr_linear (metrics/linear.py:140-215: the fp32 difference squared in
//     float64, inf when mse <= eps) and calculate_psnr (metrics/psnr.py:18-67: difference taken in float64, inf when
//     mse <= 1e-12), selected by diff_double;
//   * ssim_linear (metrics/linear.py:218-324): normalised Gaussian / uniform k x k window (separable), padding
//     reflect / replicate / circular / constant, variances clamped >= 0, ssim = num / (den + eps); the kernels return
//     the per-plane mean of the SSIM map (the caller aggregates channels and batch as the reference does).
// Reductions are fixed-order (per-block double partials, then an ordered per-sample / per-plane combine).
#include <math.h>

#include "nbp_common.h"

using namespace nbp;

namespace {

__global__ __launch_bounds__(256) void sqerr_kernel(const float* __restrict__ a, const float* __restrict__ b, long L,
                                                    int chunks, int diff_double, double* __restrict__ slab) {
  __shared__ double red[16];
  const int n = blockIdx.y;
  const long per = (L + chunks - 1) / chunks, l0 = (long)blockIdx.x * per, l1 = min(L, l0 + per);
  const float* pa = a + (long)n * L;
  const float* pb = b + (long)n * L;
  double acc = 0.0;
  for (long i = l0 + threadIdx.x; i < l1; i += blockDim.x) {
    const double d = diff_double ? (double)pa[i] - (double)pb[i] : (double)(pa[i] - pb[i]);
    acc += d * d;
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) slab[(long)n * chunks + blockIdx.x] = t;
}

__global__ void psnr_finalize(const double* __restrict__ slab, int N, int chunks, long L, double data_range,
                              double eps, double* __restrict__ mse_out, double* __restrict__ psnr_out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += slab[(long)n * chunks + c];
  const double mse = s / (double)L;
  if (mse_out) mse_out[n] = mse;
  psnr_out[n] = mse <= eps ? INFINITY : 10.0 * log10((data_range * data_range) / fmax(mse, eps));
}

enum { PAD_REFLECT = 0, PAD_REPLICATE = 1, PAD_CIRCULAR = 2, PAD_CONSTANT = 3 };

// index into [0, n) of the padded coordinate i (may be out of range); -1 = zero (constant padding)
__device__ __forceinline__ int pad_index(int i, int n, int mode) {
  if (i >= 0 && i < n) return i;
  switch (mode) {
    case PAD_REFLECT: return i < 0 ? -i : 2 * (n - 1) - i;
    case PAD_REPLICATE: return i < 0 ? 0 : n - 1;
    case PAD_CIRCULAR: return ((i % n) + n) % n;
    default: return -1;
  }
}

// horizontal pass: hb[q][p][i][j] = sum_t w[t] f_q(row i, column j + t - r), q over {x, y, xx, yy, xy}
__global__ __launch_bounds__(256) void ssim_lin_h(const float* __restrict__ x, const float* __restrict__ y,
                                                  const float* __restrict__ w, int k, long planes, int H, int W,
                                                  int mode, float* __restrict__ hb) {
  const long total = planes * H * W;
  const int r = k / 2;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int j = e % W;
    const long row = e / W;  // plane * H + i
    const float* xr = x + row * W;
    const float* yr = y + row * W;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
    for (int t = 0; t < k; ++t) {
      const int jj = pad_index(j + t - r, W, mode);
      if (jj < 0) continue;
      const float a = xr[jj], b = yr[jj], wt = w[t];
      s0 = fmaf(wt, a, s0);
      s1 = fmaf(wt, b, s1);
      s2 = fmaf(wt, a * a, s2);
      s3 = fmaf(wt, b * b, s3);
      s4 = fmaf(wt, a * b, s4);
    }
    hb[e] = s0;
    hb[total + e] = s1;
    hb[2 * total + e] = s2;
    hb[3 * total + e] = s3;
    hb[4 * total + e] = s4;
  }
}

// vertical pass + SSIM map + per-(plane, chunk) partial sums
// clamp_var: variances clamped >= 0 (linear.py); crop: only pixels at distance >= k/2 from the border are averaged
// (torchmetrics crops the padded border of the SSIM map)
__global__ __launch_bounds__(256) void ssim_lin_v(const float* __restrict__ hb, const float* __restrict__ w, int k,
                                                  long planes, int H, int W, int mode, float c1, float c2, float eps,
                                                  int clamp_var, int crop, int chunks, double* __restrict__ slab) {
  __shared__ double red[16];
  const long total = planes * H * W;
  const int p = blockIdx.y, r = k / 2;
  const long HW = (long)H * W;
  const long per = (HW + chunks - 1) / chunks, q0 = (long)blockIdx.x * per, q1 = min(HW, q0 + per);
  double acc = 0.0;
  for (long q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
    const int i = q / W, j = q - (long)i * W;
    if (crop && (i < r || i >= H - r || j < r || j >= W - r)) continue;
    float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < k; ++t) {
      const int ii = pad_index(i + t - r, H, mode);
      if (ii < 0) continue;
      const long o = (long)p * HW + (long)ii * W + j;
      const float wt = w[t];
#pragma unroll
      for (int c = 0; c < 5; ++c) m[c] = fmaf(wt, hb[c * total + o], m[c]);
    }
    const float mx2 = m[0] * m[0], my2 = m[1] * m[1], mxy = m[0] * m[1];
    float sx = m[2] - mx2, sy = m[3] - my2;
    const float sxy = m[4] - mxy;
    if (clamp_var) {
      sx = fmaxf(sx, 0.f);
      sy = fmaxf(sy, 0.f);
    }
    const float num = (2.f * m[0] * m[1] + c1) * (2.f * sxy + c2);
    const float den = (mx2 + my2 + c1) * (sx + sy + c2);
    acc += (double)(num / (den + eps));
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) slab[(long)p * chunks + blockIdx.x] = t;
}

__global__ void plane_mean_finalize(const double* __restrict__ slab, long P, int chunks, double inv,
                                    double* __restrict__ out) {
  const long p = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (p >= P) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += slab[p * chunks + c];
  out[p] = s * inv;
}

inline int chunks_for(long per_item, long items) {
  long c = (per_item + 4095) / 4096;  // >= 4096 elements per block
  long want = (2048 + items - 1) / items;
  if (c > want) c = want;
  if (c < 1) c = 1;
  if (c > 1024) c = 1024;
  return (int)c;
}

// |sobel(L)| with zero padding (F.conv2d(l, K, padding=1), color_error.py:296-302): sqrt(gx^2 + gy^2 + 1e-12)
__global__ __launch_bounds__(256) void sobel_mag_kernel(const float* __restrict__ lab, long HW, int H, int W, long npix,
                                                        float* __restrict__ out) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const int i = q / W, j = q - (long)i * W;
    const float* L = lab + b * 3 * HW;  // channel 0 of [B][3][H][W]
    auto at = [&](int y, int x) { return (y < 0 || y >= H || x < 0 || x >= W) ? 0.f : L[(long)y * W + x]; };
    // cross-correlation with Kx = [[-1,0,1],[-2,0,2],[-1,0,1]], Ky = Kx^T
    const float gx = -at(i - 1, j - 1) + at(i - 1, j + 1) - 2.f * at(i, j - 1) + 2.f * at(i, j + 1) - at(i + 1, j - 1) +
                     at(i + 1, j + 1);
    const float gy = -at(i - 1, j - 1) - 2.f * at(i - 1, j) - at(i - 1, j + 1) + at(i + 1, j - 1) + 2.f * at(i + 1, j) +
                     at(i + 1, j + 1);
    out[p] = sqrtf(gx * gx + gy * gy + 1e-12f);
  }
}

}  // namespace

// ---------------------------------------------------------------- calculate_ssim input alignment (metrics/ssim.py)
// BT.601 luma (ssim.py:119-131): y = 0.2989 r + 0.5870 g + 0.1140 b, evaluated as torch does it (each product and
// each sum rounded to fp32 on its own: no contraction), NCHW [N,3,H,W] -> [N,1,H,W]
__global__ __launch_bounds__(256) void luma_bt601_kernel(const float* __restrict__ x, long HW, long npix,
                                                         float* __restrict__ y) {
#pragma clang fp contract(off)  // no FMA: torch rounds each product and each sum
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const float* xb = x + b * 3 * HW + q;
    const float t = 0.2989f * xb[0] + 0.5870f * xb[HW];
    y[p] = t + 0.1140f * xb[2 * HW];
  }
}

// F.interpolate(mode='bilinear' | 'bicubic', align_corners=False) of NCHW planes (ssim.py:144-152, resize_policy
// 'resize'), torch's CPU formulas (aten UpSample.h): scale = in / out, src = scale * (dst + 0.5) - 0.5; bilinear clamps
// src at 0, taps i0 = min(floor(src), in - 1), i1 = i0 + (i0 < in - 1), weights 1 - l, l; bicubic: taps floor(src) - 1
// .. + 2 clamped to the border, Keys' kernel A = -0.75.
__device__ __forceinline__ void cubic_coeffs(float t, float c[4]) {
  const float A = -0.75f;
  auto cc1 = [&](float x) { return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f; };        // |x| <= 1
  auto cc2 = [&](float x) { return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A; };  // 1 < |x| < 2
  c[0] = cc2(t + 1.f);
  c[1] = cc1(t);
  c[2] = cc1(1.f - t);
  c[3] = cc2((1.f - t) + 1.f);
}

template <bool CUBIC>
__global__ __launch_bounds__(256) void resize_kernel(const float* __restrict__ x, int Hi, int Wi, int Ho, int Wo,
                                                     long total, float sh, float sw, float* __restrict__ y) {
#pragma clang fp contract(off)  // torch's CPU loops round every product and sum
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int ow = (int)(e % Wo);
    const long t = e / Wo;
    const int oh = (int)(t % Ho);
    const long plane = t / Ho;
    const float* xp = x + plane * Hi * Wi;
    const float rh = sh * (oh + 0.5f) - 0.5f, rw = sw * (ow + 0.5f) - 0.5f;
    if (!CUBIC) {
      const float fh = fmaxf(rh, 0.f), fw = fmaxf(rw, 0.f);
      const int h0 = min((int)floorf(fh), Hi - 1), w0 = min((int)floorf(fw), Wi - 1);
      const int h1 = h0 + (h0 < Hi - 1 ? 1 : 0), w1 = w0 + (w0 < Wi - 1 ? 1 : 0);
      const float lh = fminf(fmaxf(fh - h0, 0.f), 1.f), lw = fminf(fmaxf(fw - w0, 0.f), 1.f);
      const float top = (1.f - lw) * xp[(long)h0 * Wi + w0] + lw * xp[(long)h0 * Wi + w1];
      const float bot = (1.f - lw) * xp[(long)h1 * Wi + w0] + lw * xp[(long)h1 * Wi + w1];
      y[e] = (1.f - lh) * top + lh * bot;
    } else {
      const int h0 = (int)floorf(rh), w0 = (int)floorf(rw);
      float ch[4], cw[4];
      cubic_coeffs(rh - h0, ch);
      cubic_coeffs(rw - w0, cw);
      float acc = 0.f;
      for (int i = 0; i < 4; ++i) {
        const int hh = min(max(h0 - 1 + i, 0), Hi - 1);
        float row = 0.f;
        for (int j = 0; j < 4; ++j) row += cw[j] * xp[(long)hh * Wi + min(max(w0 - 1 + j, 0), Wi - 1)];
        acc += ch[i] * row;
      }
      y[e] = acc;
    }
  }
}

extern "C" {

int nbp_sobel_mag(const float* lab, int B, int H, int W, float* out, nbp_stream_t s) {
  NBP_REQUIRE(lab && out && B > 0 && H > 0 && W > 0, "nbp_sobel_mag: bad args");
  const long HW = (long)H * W, n = B * HW;
  long g = (n + 255) / 256;
  sobel_mag_kernel<<<(int)(g > 8192 ? 8192 : g), 256, 0, S(s)>>>(lab, HW, H, W, n, out);
  return check_launch("sobel_mag");
}

size_t nbp_psnr_workspace_doubles(int N, long L) { return (size_t)N * chunks_for(L, N); }

int nbp_psnr(const float* pred, const float* tgt, int N, long L, double data_range, double eps, int diff_double,
             double* ws, double* mse, double* psnr, nbp_stream_t s) {
  NBP_REQUIRE(pred && tgt && ws && psnr && N > 0 && L > 0 && N <= 65535, "nbp_psnr: bad args");
  NBP_REQUIRE(data_range > 0.0, "nbp_psnr: data_range must be positive");
  const int chunks = chunks_for(L, N);
  sqerr_kernel<<<dim3(chunks, N), 256, 0, S(s)>>>(pred, tgt, L, chunks, diff_double, ws);
  psnr_finalize<<<cdiv(N, 256), 256, 0, S(s)>>>(ws, N, chunks, L, data_range, eps, mse, psnr);
  return check_launch("psnr");
}

size_t nbp_ssim_linear_workspace_floats(int N, int C, int H, int W) {
  const long P = (long)N * C, HW = (long)H * W;
  return (size_t)5 * P * HW + 2 * (size_t)P * chunks_for(HW, P);  // 5 filtered maps + the double slab
}

int nbp_ssim_linear(const float* pred, const float* tgt, int N, int C, int H, int W, const float* win, int k,
                    int pad_mode, float c1, float c2, float eps, int clamp_var, int crop, float* ws, double* out,
                    nbp_stream_t s) {
  NBP_REQUIRE(pred && tgt && win && ws && out && N > 0 && C > 0 && H > 0 && W > 0, "nbp_ssim_linear: bad args");
  NBP_REQUIRE(k > 0 && k % 2 == 1 && H >= k && W >= k, "nbp_ssim_linear: odd window no larger than the image");
  NBP_REQUIRE(pad_mode >= 0 && pad_mode <= 3, "nbp_ssim_linear: pad_mode");
  NBP_REQUIRE(!crop || (H > 2 * (k / 2) && W > 2 * (k / 2)), "nbp_ssim_linear: nothing left after the crop");
  NBP_REQUIRE((long)N * C <= 65535, "nbp_ssim_linear: too many planes");
  const long P = (long)N * C, HW = (long)H * W, total = P * HW;
  const int chunks = chunks_for(HW, P);
  float* hb = ws;
  double* slab = reinterpret_cast<double*>(ws + 5 * total + ((5 * total) & 1));  // 8-byte aligned
  long g = (total + 255) / 256;
  ssim_lin_h<<<(int)(g > 8192 ? 8192 : g), 256, 0, S(s)>>>(pred, tgt, win, k, P, H, W, pad_mode, hb);
  ssim_lin_v<<<dim3(chunks, P), 256, 0, S(s)>>>(hb, win, k, P, H, W, pad_mode, c1, c2, eps, clamp_var, crop, chunks,
                                                 slab);
  const long r = k / 2, cnt = crop ? (long)(H - 2 * r) * (W - 2 * r) : HW;
  plane_mean_finalize<<<cdiv(P, 256), 256, 0, S(s)>>>(slab, P, chunks, 1.0 / (double)cnt, out);
  return check_launch("ssim_linear");
}

int nbp_luma_bt601(const float* x, int N, int H, int W, float* y, nbp_stream_t s) {
  NBP_REQUIRE(x && y && N > 0 && H > 0 && W > 0, "nbp_luma_bt601: bad args");
  const long HW = (long)H * W, n = (long)N * HW;
  long g = (n + 255) / 256;
  luma_bt601_kernel<<<(int)(g > 8192 ? 8192 : g), 256, 0, S(s)>>>(x, HW, n, y);
  return check_launch("luma_bt601");
}

int nbp_resize_planes(const float* x, long planes, int Hi, int Wi, int Ho, int Wo, int cubic, float* y, nbp_stream_t s) {
  NBP_REQUIRE(x && y && planes > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "nbp_resize_planes: bad args");
  const long total = planes * Ho * Wo;
  long g = (total + 255) / 256;
  const int grid = (int)(g > 8192 ? 8192 : g);
  const float sh = (float)Hi / (float)Ho, sw = (float)Wi / (float)Wo;
  if (cubic) resize_kernel<true><<<grid, 256, 0, S(s)>>>(x, Hi, Wi, Ho, Wo, total, sh, sw, y);
  else resize_kernel<false><<<grid, 256, 0, S(s)>>>(x, Hi, Wi, Ho, Wo, total, sh, sw, y);
  return check_launch("resize_planes");
}

}  // extern "C"
