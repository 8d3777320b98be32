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

// ---------------------------------------------------------------- SSIM, LDS-tiled (one launch forward, one backward)
// Forward: a TH x TW output tile of one plane.  x, y (clamped) are staged with a 5-pixel halo at reflected
// coordinates (reflect padding = the reflected pixel itself), the horizontal 11-tap pass of {x, y, x^2, y^2, xy}
// runs LDS -> LDS, the vertical pass LDS -> registers, then the SSIM map, the per-block loss partial and the three
// gradient-coefficient maps (the only global writes).  Every input pixel is read from HBM once (+halo).
constexpr int SS_TH = 32, SS_TW = 64, SS_R = 5;

// inv_n: the reduction's weight of one pixel in the coefficient maps (1/n for 'mean', 1 for 'sum' and 'none'; with
// 'none' the backward multiplies each coefficient by that pixel's upstream gradient); lmap (optional): the clamped
// per-pixel loss map (reduction 'none')
__global__ __launch_bounds__(256) void ssim_fwd_tiled(const float* __restrict__ x, const float* __restrict__ y, int H,
                                                       int W, int clamp_in, Win win, float C1, float C2, float eps,
                                                       float inv_n, double* __restrict__ partial,
                                                       float* __restrict__ coef, float* __restrict__ lmap, long n) {
  constexpr int LH = SS_TH + 2 * SS_R, LW = SS_TW + 2 * SS_R;
  __shared__ float xs[LH][LW + 1], ys[LH][LW + 1];
  __shared__ float hm[5][LH][SS_TW + 1];
  __shared__ double red[16];
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * SS_TW, y0 = blockIdx.y * SS_TH;
  const long plane = blockIdx.z;
  const float* xp = x + plane * H * W;
  const float* yp = y + plane * H * W;
  // staging in batches of 4 positions per thread: all 8 loads issued before the LDS stores
  for (int e0 = tid; e0 < LH * LW; e0 += 4 * 256) {
    float xv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256;
      const int r = e / LW, c = e % LW;
      const int gy = y0 - SS_R + r, gx = x0 - SS_R + c;
      xv[u] = yv[u] = 0.f;
      if (e < LH * LW && gy < H + SS_R && gx < W + SS_R) {  // positions further out feed no valid output
        const long o = (long)refl(gy, H) * W + refl(gx, W);
        xv[u] = xp[o];
        yv[u] = yp[o];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256;
      if (e >= LH * LW) break;
      const int r = e / LW, c = e % LW;
      xs[r][c] = clamp_in ? clamp01(xv[u]) : xv[u];
      ys[r][c] = clamp_in ? clamp01(yv[u]) : yv[u];
    }
  }
  __syncthreads();
  for (int e = tid; e < LH * SS_TW; e += 256) {
    const int r = e / SS_TW, c = e % SS_TW;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
    for (int t = 0; t < 11; ++t) {
      const float xv = xs[r][c + t], yv = ys[r][c + t], k = win.k[t];
      s0 = fmaf(k, xv, s0);
      s1 = fmaf(k, yv, s1);
      s2 = fmaf(k, xv * xv, s2);
      s3 = fmaf(k, yv * yv, s3);
      s4 = fmaf(k, xv * yv, s4);
    }
    hm[0][r][c] = s0; hm[1][r][c] = s1; hm[2][r][c] = s2; hm[3][r][c] = s3; hm[4][r][c] = s4;
  }
  __syncthreads();
  double sacc = 0.0;
  for (int e = tid; e < SS_TH * SS_TW; e += 256) {
    const int r = e / SS_TW, c = e % SS_TW;
    const int gy = y0 + r, gx = x0 + c;
    if (gy >= H || gx >= W) continue;
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 11; ++t) {
      const float k = win.k[t];
#pragma unroll
      for (int m = 0; m < 5; ++m) v[m] = fmaf(k, hm[m][r + t][c], v[m]);
    }
    const float mx = v[0], my = v[1];
    const float mx2 = mx * mx, my2 = my * my, mxy = mx * my;
    const float sxx = v[2] - mx2, syy = v[3] - my2, sxy = v[4] - mxy;
    const float A1 = 2.f * mxy + C1, A2 = 2.f * sxy + C2;
    const float B1 = mx2 + my2 + C1, B2 = sxx + syy + C2;
    const float num = A1 * A2, D = B1 * B2 + eps;
    const float S = num / D;
    const float l = (1.f - S) / 2.f;
    const float lc = fminf(fmaxf(l, 0.f), 1.f);
    sacc += lc;
    if (lmap) lmap[(plane * H + gy) * W + gx] = lc;
    if (coef) {
      const float dS = (l >= 0.f && l <= 1.f) ? -0.5f * inv_n : 0.f;
      // dnum/dmx = 2 my (A2 - A1); dden/dmx = 2 mx (B2 - B1); dS/dE[x^2] = -S B1 / D; dS/dE[xy] = 2 A1 / D
      const float dmx = (2.f * my * (A2 - A1) - S * 2.f * mx * (B2 - B1)) / D;
      const float dxx = -S * B1 / D;
      const float dxy = 2.f * A1 / D;
      const long o = (plane * H + gy) * W + gx;
      coef[o] = dS * dmx;
      coef[n + o] = dS * dxx;
      coef[2 * n + o] = dS * dxy;
    }
  }
  sacc = block_sum_d(sacc, red);
  if (tid == 0) partial[((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = sacc;
}

// Backward: gx = F^T gm + 2 x F^T gxx + y F^T gxy with F = V . H the reflect-padded separable filter, so
// F^T = H^T . V^T.  A TH x TW tile stages the three coefficient maps with a 5-pixel margin, applies the vertical
// adjoint into LDS and the horizontal adjoint from LDS; 1-D adjoint of reflect padding: output j gathers
// q in {j, -j (1 <= j <= 5), 2(n-1) - j (n-6 <= j <= n-2)}, taps q - t + 5 inside [0, n).  The reflected sources
// stay inside the margin: -j only occurs in the first tile (TH > 5) and reads rows [0, 5 - j]; 2(n-1) - j reads
// rows [n-5, n) with j >= y0.
constexpr int SB_TH = 32, SB_TW = 64, SB_M = 5;

__device__ __forceinline__ int refl_sources(int j, int n, int* qs) {
  int nq = 0;
  qs[nq++] = j;
  if (j >= 1 && j <= 5) qs[nq++] = -j;
  if (j <= n - 2 && j >= n - 6) qs[nq++] = 2 * (n - 1) - j;
  return nq;
}

// up_map (optional, reduction 'none'): the per-pixel upstream gradient, applied to the coefficients as they are
// staged (the adjoint filters are linear); otherwise the scalar up[0] scales the result
__global__ __launch_bounds__(256) void ssim_bwd_tiled(const float* __restrict__ coef, const float* __restrict__ x,
                                                       const float* __restrict__ y, int H, int W, Win win,
                                                       int clamp_in, const float* __restrict__ up,
                                                       const float* __restrict__ up_map, float* __restrict__ gx,
                                                       long n) {
  constexpr int LH = SB_TH + 2 * SB_M, LW = SB_TW + 2 * SB_M;
  __shared__ float cs[3][LH][LW + 1];
  __shared__ float tv[3][SB_TH][LW + 1];
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * SB_TW, y0 = blockIdx.y * SB_TH;
  const long plane = blockIdx.z;
  const long pb = plane * H * W;
  for (int e0 = tid; e0 < LH * LW; e0 += 4 * 256) {  // 12 loads in flight per thread, then the LDS stores
    float v[4][3];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256;
      const int r = e / LW, c = e % LW;
      const int gy = y0 - SB_M + r, gxx = x0 - SB_M + c;
      const bool in = e < LH * LW && gy >= 0 && gy < H && gxx >= 0 && gxx < W;
      const long o = pb + (long)gy * W + gxx;
      const float um = in && up_map ? up_map[o] : 1.f;
#pragma unroll
      for (int m = 0; m < 3; ++m) v[u][m] = in ? coef[m * n + o] * um : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * 256;
      if (e >= LH * LW) break;
      const int r = e / LW, c = e % LW;
#pragma unroll
      for (int m = 0; m < 3; ++m) cs[m][r][c] = v[u][m];
    }
  }
  // this thread's output pixels of x / y, loaded now so their latency overlaps the two adjoint passes
  constexpr int PER = SB_TH * SB_TW / 256;
  float xo[PER], yo[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + k * 256, r = e / SB_TW, c = e % SB_TW;
    const int j = y0 + r, i = x0 + c;
    const long o = pb + (long)j * W + i;
    const bool ok = j < H && i < W;
    xo[k] = ok ? x[o] : 0.f;
    yo[k] = ok ? y[o] : 0.f;
  }
  __syncthreads();
  // vertical adjoint for the tile's rows and every staged column
  for (int e = tid; e < SB_TH * LW; e += 256) {
    const int r = e / LW, c = e % LW;
    const int j = y0 + r;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    if (j >= 6 && j <= H - 7) {  // interior row: the plain 11-tap window, no reflected sources
      const int lb = j - (y0 - SB_M) + 5;
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const float k = win.k[t];
        a0 = fmaf(k, cs[0][lb - t][c], a0);
        a1 = fmaf(k, cs[1][lb - t][c], a1);
        a2 = fmaf(k, cs[2][lb - t][c], a2);
      }
    } else if (j < H) {
      int qs[3];
      const int nq = refl_sources(j, H, qs);
      for (int u = 0; u < nq; ++u) {
#pragma unroll
        for (int t = 0; t < 11; ++t) {
          const int rr = qs[u] - t + 5;
          if (rr < 0 || rr >= H) continue;
          const int lr = rr - (y0 - SB_M);  // inside [0, LH) by the margin
          const float k = win.k[t];
          a0 = fmaf(k, cs[0][lr][c], a0);
          a1 = fmaf(k, cs[1][lr][c], a1);
          a2 = fmaf(k, cs[2][lr][c], a2);
        }
      }
    }
    tv[0][r][c] = a0; tv[1][r][c] = a1; tv[2][r][c] = a2;
  }
  __syncthreads();
  const float g0 = up_map ? 1.f : up[0];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + k * 256;
    const int r = e / SB_TW, c = e % SB_TW;
    const int j = y0 + r, i = x0 + c;
    if (j >= H || i >= W) continue;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    if (i >= 6 && i <= W - 7) {  // interior column
      const int lb = i - (x0 - SB_M) + 5;
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const float k = win.k[t];
        a0 = fmaf(k, tv[0][r][lb - t], a0);
        a1 = fmaf(k, tv[1][r][lb - t], a1);
        a2 = fmaf(k, tv[2][r][lb - t], a2);
      }
    } else {
    int qs[3];
    const int nq = refl_sources(i, W, qs);
    for (int u = 0; u < nq; ++u) {
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const int cc = qs[u] - t + 5;
        if (cc < 0 || cc >= W) continue;
        const int lc = cc - (x0 - SB_M);
        const float k = win.k[t];
        a0 = fmaf(k, tv[0][r][lc], a0);
        a1 = fmaf(k, tv[1][r][lc], a1);
        a2 = fmaf(k, tv[2][r][lc], a2);
      }
    }
    }
    const long o = pb + (long)j * W + i;
    const float xr = xo[k];
    float xv = xr, yv = yo[k];
    if (clamp_in) { xv = clamp01(xv); yv = clamp01(yv); }
    float g = a0 + 2.f * xv * a1 + yv * a2;
    if (clamp_in && !(xr >= 0.f && xr <= 1.f)) g = 0.f;
    gx[o] = g0 * g;
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

// ws: 3 * n floats (gradient coefficients) + one double per forward block (<= n blocks)
size_t nbp_ssim_workspace_floats(long n) { return (size_t)5 * n + 4; }

int nbp_ssim_loss_fwd(const float* x, const float* y, int N, int C, int H, int W, int window, float max_val,
                      int clamp_in, int want_grad, int reduction, float* ws, float* loss, float* lmap, nbp_stream_t s) {
  NBP_REQUIRE(x && y && ws && N > 0 && C > 0 && reduction >= 0 && reduction <= 2, "nbp_ssim_loss_fwd: bad args");
  NBP_REQUIRE(reduction == 2 ? lmap != nullptr : loss != nullptr, "nbp_ssim_loss_fwd: output missing for the reduction");
  NBP_REQUIRE(window == 11, "nbp_ssim_loss_fwd: only the 11-tap window (SSIMLoss default) is implemented");
  NBP_REQUIRE(H > 5 && W > 5, "nbp_ssim_loss_fwd: reflect padding needs H, W > 5");
  NBP_REQUIRE((long)N * C <= 65535, "nbp_ssim_loss_fwd: N*C <= 65535 planes");
  const long planes = (long)N * C, n = planes * H * W;
  const Win win = make_window(11, 1.5f);
  float* coef = ws;
  double* partial = reinterpret_cast<double*>(ws + 3 * n + ((3 * n) & 1));
  const dim3 g(cdiv(W, SS_TW), cdiv(H, SS_TH), (unsigned)planes);
  const int nb = (int)(g.x * g.y * g.z);
  const float C1 = (0.01f * max_val) * (0.01f * max_val), C2 = (0.03f * max_val) * (0.03f * max_val);
  const float inv_n = reduction == 0 ? (float)(1.0 / (double)n) : 1.f;
  ssim_fwd_tiled<<<g, 256, 0, S(s)>>>(x, y, H, W, clamp_in, win, C1, C2, 1e-12f, inv_n, partial,
                                      want_grad ? coef : nullptr, reduction == 2 ? lmap : nullptr, n);
  if (loss) finalize_mean<<<1, 256, 0, S(s)>>>(partial, nb, reduction == 0 ? 1.0 / (double)n : 1.0, loss);
  return check_launch("ssim_loss_fwd");
}

// requires the workspace of a forward call made with want_grad = 1 on the same inputs
int nbp_ssim_loss_bwd(const float* x, const float* y, int N, int C, int H, int W, int clamp_in, const float* up,
                      const float* up_map, float* ws, float* gx, nbp_stream_t s) {
  NBP_REQUIRE(x && y && ws && (up || up_map) && gx && N > 0 && C > 0 && H > 5 && W > 5, "nbp_ssim_loss_bwd: bad args");
  NBP_REQUIRE((long)N * C <= 65535, "nbp_ssim_loss_bwd: N*C <= 65535 planes");
  const long planes = (long)N * C, n = planes * H * W;
  const Win win = make_window(11, 1.5f);
  const dim3 g(cdiv(W, SB_TW), cdiv(H, SB_TH), (unsigned)planes);
  ssim_bwd_tiled<<<g, 256, 0, S(s)>>>(ws, x, y, H, W, win, clamp_in, up, up_map, gx, n);
  return check_launch("ssim_loss_bwd");
}

}  // extern "C"
