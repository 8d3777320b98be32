// HybridLoss pixel/structure terms on NCHW images:
//   L1 (nn.L1Loss, NewBP_model/losses.py:249,332) and Charbonnier (basicsr losses.py:29-31, sqrt(d^2 + eps));
//   SSIMLoss (losses.py:146-155 -> kornia 0.6.12 ssim_loss: 11x11 Gaussian sigma 1.5, reflect padding,
//   C1=(0.01L)^2, C2=(0.03L)^2, loss = mean(clamp((1 - ssim)/2, 0, 1))) with its analytic gradient w.r.t. the
//   prediction.  The 2-D window is applied as two 1-D passes (it is an outer product); the backward applies the
//   adjoint of each reflect-padded 1-D pass.
#include <math.h>

#include "nbp_common.h"

using namespace nbp;

namespace {

struct Win {
  float k[11];
};

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }
__device__ __forceinline__ int refl(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * (n - 1) - i;
  return i;
}

// mode 0: |d| ; mode 1: sqrt(d^2 + eps)
__global__ void pix_fwd(const float* __restrict__ a, const float* __restrict__ b, long n, int mode, float eps,
                        int clamp_a, int clamp_b, double* __restrict__ partial) {
  __shared__ double red[16];
  double s = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float av = a[i], bv = b[i];
    if (clamp_a) av = clamp01(av);
    if (clamp_b) bv = clamp01(bv);
    const float d = av - bv;
    s += mode == 0 ? fabsf(d) : sqrtf(d * d + eps);
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void pix_bwd(const float* __restrict__ a, const float* __restrict__ b, long n, int mode, float eps,
                        int clamp_a, int clamp_b, const float* __restrict__ up, float scale, float* __restrict__ ga) {
  const float g0 = up[0] * scale;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float ar = a[i];
    float av = ar, bv = b[i];
    if (clamp_a) av = clamp01(av);
    if (clamp_b) bv = clamp01(bv);
    const float d = av - bv;
    float g = mode == 0 ? (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) : d / sqrtf(d * d + eps);
    if (clamp_a && !(ar >= 0.f && ar <= 1.f)) g = 0.f;
    ga[i] = g0 * g;
  }
}

__global__ void finalize_mean(const double* __restrict__ partial, int n, double scale, float* __restrict__ out) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) out[0] = (float)(s * scale);
}

// pass 1: horizontal filter of {x, y, x^2, y^2, xy} (clamped inputs) into h[5][plane][H][W]
// (all SSIM kernels: planes * H * W < 2^31, checked on the host: 32-bit index arithmetic, 64-bit map offsets)
__global__ void ssim_h(const float* __restrict__ x, const float* __restrict__ y, float* __restrict__ hbuf, long planes,
                       int H, int W, int clamp_in, Win win) {
  const int total = (int)(planes * H * W);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W;
    const int row = i / W;
    const float* xr = x + (long)row * W;
    const float* yr = y + (long)row * W;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
    for (int t = 0; t < 11; ++t) {
      const int c = refl(w + t - 5, W);
      float xv = xr[c], yv = yr[c];
      if (clamp_in) { xv = clamp01(xv); yv = clamp01(yv); }
      const float k = win.k[t];
      s0 = fmaf(k, xv, s0);
      s1 = fmaf(k, yv, s1);
      s2 = fmaf(k, xv * xv, s2);
      s3 = fmaf(k, yv * yv, s3);
      s4 = fmaf(k, xv * yv, s4);
    }
    const long tl = total;
    hbuf[i] = s0;
    hbuf[tl + i] = s1;
    hbuf[2 * tl + i] = s2;
    hbuf[3 * tl + i] = s3;
    hbuf[4 * tl + i] = s4;
  }
}

// pass 2: vertical filter -> ssim map -> loss partials and the three gradient coefficient maps
//   gm = dL/dmu_x, gxx = dL/dE[x^2], gxy = dL/dE[xy]   (dL/dS = -0.5 * inv_n inside the clamp window)
__global__ void ssim_v(const float* __restrict__ hbuf, long planes, int H, int W, Win win, float C1, float C2, float eps,
                       float inv_n, double* __restrict__ partial, float* __restrict__ coef) {
  __shared__ double red[16];
  const int total = (int)(planes * H * W);
  const long tl = total;
  double s = 0.0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W;
    const int h = hw % H;
    const int plane = hw / H;
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 11; ++t) {
      const int o = (plane * H + refl(h + t - 5, H)) * W + w;
      const float k = win.k[t];
#pragma unroll
      for (int j = 0; j < 5; ++j) v[j] = fmaf(k, hbuf[j * tl + o], v[j]);
    }
    const float mx = v[0], my = v[1];
    const float mx2 = mx * mx, my2 = my * my, mxy = mx * my;
    const float sxx = v[2] - mx2, syy = v[3] - my2, sxy = v[4] - mxy;
    const float A1 = 2.f * mxy + C1, A2 = 2.f * sxy + C2;
    const float B1 = mx2 + my2 + C1, B2 = sxx + syy + C2;
    const float num = A1 * A2, D = B1 * B2 + eps;
    const float S = num / D;
    const float l = (1.f - S) / 2.f;
    s += fminf(fmaxf(l, 0.f), 1.f);
    if (coef) {
      const float dS = (l >= 0.f && l <= 1.f) ? -0.5f * inv_n : 0.f;
      // dnum/dmx = 2 my (A2 - A1); dden/dmx = 2 mx (B2 - B1); dS/dE[x^2] = -S B1 / D; dS/dE[xy] = 2 A1 / D
      const float dmx = (2.f * my * (A2 - A1) - S * 2.f * mx * (B2 - B1)) / D;
      const float dxx = -S * B1 / D;
      const float dxy = 2.f * A1 / D;
      coef[i] = dS * dmx;
      coef[tl + i] = dS * dxx;
      coef[2 * tl + i] = dS * dxy;
    }
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// adjoint of one reflect-padded 1-D pass along rows (vertical) for three maps: out[j] = sum_{q->j} sum_t k[t] in[q-t+5]
__global__ void ssim_vT(const float* __restrict__ coef, float* __restrict__ tbuf, long planes, int H, int W, Win win) {
  const int total = (int)(planes * H * W);
  const long tl = total;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int w = i % W, hw = i / W;
    const int j = hw % H;
    const int plane = hw / H;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    int qs[3];
    int nq = 0;
    qs[nq++] = j;
    if (j >= 1 && j <= 5) qs[nq++] = -j;
    if (j <= H - 2 && j >= H - 6) qs[nq++] = 2 * (H - 1) - j;
    for (int u = 0; u < nq; ++u) {
      const int q = qs[u];
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const int r = q - t + 5;
        if (r < 0 || r >= H) continue;
        const int o = (plane * H + r) * W + w;
        const float k = win.k[t];
        a0 = fmaf(k, coef[o], a0);
        a1 = fmaf(k, coef[tl + o], a1);
        a2 = fmaf(k, coef[2 * tl + o], a2);
      }
    }
    tbuf[i] = a0;
    tbuf[tl + i] = a1;
    tbuf[2 * tl + i] = a2;
  }
}

// adjoint along columns, then combine: gx = F^T gm + 2 x F^T gxx + y F^T gxy  (x, y clamped; clamp mask on x)
__global__ void ssim_hT(const float* __restrict__ tbuf, const float* __restrict__ x, const float* __restrict__ y,
                        long planes, int H, int W, Win win, int clamp_in, const float* __restrict__ up,
                        float* __restrict__ gx) {
  const int total = (int)(planes * H * W);
  const long tl = total;
  const float g0 = up[0];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = i % W;
    const int row = i / W;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    int qs[3];
    int nq = 0;
    qs[nq++] = j;
    if (j >= 1 && j <= 5) qs[nq++] = -j;
    if (j <= W - 2 && j >= W - 6) qs[nq++] = 2 * (W - 1) - j;
    for (int u = 0; u < nq; ++u) {
      const int q = qs[u];
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const int c = q - t + 5;
        if (c < 0 || c >= W) continue;
        const int o = row * W + c;
        const float k = win.k[t];
        a0 = fmaf(k, tbuf[o], a0);
        a1 = fmaf(k, tbuf[tl + o], a1);
        a2 = fmaf(k, tbuf[2 * tl + o], a2);
      }
    }
    const float xr = x[i];
    float xv = xr, yv = y[i];
    if (clamp_in) { xv = clamp01(xv); yv = clamp01(yv); }
    float g = a0 + 2.f * xv * a1 + yv * a2;
    if (clamp_in && !(xr >= 0.f && xr <= 1.f)) g = 0.f;
    gx[i] = g0 * g;
  }
}

inline int grid_for(long total) {
  long g = (total + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

Win make_window(int ks, float sigma) {
  // kornia gaussian(): x = arange(ks) - ks//2, exp(-x^2 / (2 sigma^2)), normalised by its sum (fp32)
  Win w{};
  float s = 0.f;
  for (int i = 0; i < ks; ++i) {
    const float x = (float)(i - ks / 2);
    w.k[i] = expf(-(x * x) / (2.f * sigma * sigma));
    s += w.k[i];
  }
  for (int i = 0; i < ks; ++i) w.k[i] /= s;
  return w;
}

}  // namespace

extern "C" {

size_t nbp_pix_workspace_doubles(long n) { return (size_t)grid_for(n); }

int nbp_pix_loss_fwd(const float* a, const float* b, long n, int mode, float eps, int clamp_a, int clamp_b, double* ws,
                     float* loss, nbp_stream_t s) {
  NBP_REQUIRE(a && b && ws && loss && n > 0 && (mode == 0 || mode == 1), "nbp_pix_loss_fwd: bad args");
  const int g = grid_for(n);
  pix_fwd<<<g, 256, 0, S(s)>>>(a, b, n, mode, eps, clamp_a, clamp_b, ws);
  finalize_mean<<<1, 256, 0, S(s)>>>(ws, g, 1.0 / (double)n, loss);
  return check_launch("pix_loss_fwd");
}

int nbp_pix_loss_bwd(const float* a, const float* b, long n, int mode, float eps, int clamp_a, int clamp_b,
                     const float* up, float* ga, nbp_stream_t s) {
  NBP_REQUIRE(a && b && up && ga && n > 0, "nbp_pix_loss_bwd: bad args");
  pix_bwd<<<grid_for(n), 256, 0, S(s)>>>(a, b, n, mode, eps, clamp_a, clamp_b, up, (float)(1.0 / (double)n), ga);
  return check_launch("pix_loss_bwd");
}

// ws: 5 * n floats (filtered maps) + 3 * n (coefficients) + grid doubles
size_t nbp_ssim_workspace_floats(long n) { return (size_t)8 * n + 2 * (size_t)grid_for(n) + 2; }

int nbp_ssim_loss_fwd(const float* x, const float* y, int N, int C, int H, int W, int window, float max_val,
                      int clamp_in, int want_grad, float* ws, float* loss, nbp_stream_t s) {
  NBP_REQUIRE(x && y && ws && loss && N > 0 && C > 0, "nbp_ssim_loss_fwd: bad args");
  NBP_REQUIRE(window == 11, "nbp_ssim_loss_fwd: only the 11-tap window (SSIMLoss default) is implemented");
  NBP_REQUIRE(H > 5 && W > 5, "nbp_ssim_loss_fwd: reflect padding needs H, W > 5");
  NBP_REQUIRE((long)N * C * H * W < (1L << 31), "nbp_ssim_loss_fwd: N*C*H*W must be < 2^31");
  const long planes = (long)N * C, n = planes * H * W;
  const Win win = make_window(11, 1.5f);
  float* hbuf = ws;
  float* coef = ws + 5 * n;
  double* partial = reinterpret_cast<double*>(ws + 8 * n + ((8 * n) & 1));
  const int g = grid_for(n);
  const float C1 = (0.01f * max_val) * (0.01f * max_val), C2 = (0.03f * max_val) * (0.03f * max_val);
  ssim_h<<<g, 256, 0, S(s)>>>(x, y, hbuf, planes, H, W, clamp_in, win);
  ssim_v<<<g, 256, 0, S(s)>>>(hbuf, planes, H, W, win, C1, C2, 1e-12f, (float)(1.0 / (double)n), partial,
                               want_grad ? coef : nullptr);
  finalize_mean<<<1, 256, 0, S(s)>>>(partial, g, 1.0 / (double)n, loss);
  return check_launch("ssim_loss_fwd");
}

// requires the workspace of a forward call made with want_grad = 1 on the same inputs
int nbp_ssim_loss_bwd(const float* x, const float* y, int N, int C, int H, int W, int clamp_in, const float* up,
                      float* ws, float* gx, nbp_stream_t s) {
  NBP_REQUIRE(x && y && ws && up && gx && N > 0 && C > 0 && H > 5 && W > 5, "nbp_ssim_loss_bwd: bad args");
  NBP_REQUIRE((long)N * C * H * W < (1L << 31), "nbp_ssim_loss_bwd: N*C*H*W must be < 2^31");
  const long planes = (long)N * C, n = planes * H * W;
  const Win win = make_window(11, 1.5f);
  float* tbuf = ws;  // reuse the filtered-map space
  const float* coef = ws + 5 * n;
  const int g = grid_for(n);
  ssim_vT<<<g, 256, 0, S(s)>>>(coef, tbuf, planes, H, W, win);
  ssim_hT<<<g, 256, 0, S(s)>>>(tbuf, x, y, planes, H, W, win, clamp_in, up, gx);
  return check_launch("ssim_loss_bwd");
}

}  // extern "C"
