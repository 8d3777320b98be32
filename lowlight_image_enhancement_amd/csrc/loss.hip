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
// Both passes are register-blocked by 4 along their filter direction: a thread reads the 14 staged values four
// outputs need once and runs each output's 11-tap chain in the original tap order (so every coefficient is bitwise the
// unblocked kernel's); the horizontal passes read LDS as float4 (row pitch 76, a multiple of 4).
constexpr int SS_P = SS_TW + 2 * SS_R + 2;

// inv_n: the reduction's weight of one pixel in the coefficient maps (1/n for 'mean', 1 for 'sum' and 'none'; with
// 'none' the backward multiplies each coefficient by that pixel's upstream gradient); lmap (optional): the clamped
// per-pixel loss map (reduction 'none')
__global__ __launch_bounds__(256) void ssim_fwd_tiled(const float* __restrict__ x, const float* __restrict__ y, int H,
                                                       int W, int clamp_in, Win win, float C1, float C2, float eps,
                                                       float inv_n, double* __restrict__ partial,
                                                       float* __restrict__ coef, float* __restrict__ lmap, long n) {
  constexpr int LH = SS_TH + 2 * SS_R, LW = SS_TW + 2 * SS_R;
  // hm (the horizontal pass) overwrites xs / ys once every task holds its outputs in registers: 54 KB of LDS per
  // tile, three tiles per CU
  static_assert(5 * SS_TW >= 2 * SS_P, "hm must cover xs / ys");
  __shared__ __attribute__((aligned(16))) float sbuf[5 * LH * SS_TW];
  auto xs = reinterpret_cast<float (*)[SS_P]>(sbuf);
  auto ys = reinterpret_cast<float (*)[SS_P]>(sbuf + LH * SS_P);
  auto hm = reinterpret_cast<float (*)[LH][SS_TW]>(sbuf);
  __shared__ double red[16];
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * SS_TW, y0 = blockIdx.y * SS_TH;
  const long plane = blockIdx.z;
  const float* xp = x + plane * H * W;
  const float* yp = y + plane * H * W;
  // staging: every load of the thread's NB positions issued before the first LDS store
  constexpr int NB = (LH * LW + 255) / 256;
  float xv[NB], yv[NB];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int e = tid + u * 256;
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
  for (int u = 0; u < NB; ++u) {
    const int e = tid + u * 256;
    if (e >= LH * LW) break;
    const int r = e / LW, c = e % LW;
    xs[r][c] = clamp_in ? clamp01(xv[u]) : xv[u];
    ys[r][c] = clamp_in ? clamp01(yv[u]) : yv[u];
  }
  __syncthreads();
  // horizontal 11-tap pass of {x, y, x^2, y^2, xy}: one row, four consecutive output columns per task
  constexpr int HT = LH * (SS_TW / 4), HIT = (HT + 255) / 256;
  float o[HIT][5][4];
#pragma unroll
  for (int it = 0; it < HIT; ++it) {
    const int e = tid + it * 256;
    if (e >= HT) break;
    const int r = e >> 4, c0 = (e & 15) * 4;
    float xw[16], yw[16];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const float4 a = *reinterpret_cast<const float4*>(&xs[r][c0 + 4 * s4]);
      const float4 b = *reinterpret_cast<const float4*>(&ys[r][c0 + 4 * s4]);
      xw[4 * s4] = a.x; xw[4 * s4 + 1] = a.y; xw[4 * s4 + 2] = a.z; xw[4 * s4 + 3] = a.w;
      yw[4 * s4] = b.x; yw[4 * s4 + 1] = b.y; yw[4 * s4 + 2] = b.z; yw[4 * s4 + 3] = b.w;
    }
    float xx[14], yy[14], xy[14];  // the products once per staged value, not once per tap
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      xx[i] = xw[i] * xw[i];
      yy[i] = yw[i] * yw[i];
      xy[i] = xw[i] * yw[i];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const float k = win.k[t];
        s0 = fmaf(k, xw[q + t], s0);
        s1 = fmaf(k, yw[q + t], s1);
        s2 = fmaf(k, xx[q + t], s2);
        s3 = fmaf(k, yy[q + t], s3);
        s4 = fmaf(k, xy[q + t], s4);
      }
      o[it][0][q] = s0; o[it][1][q] = s1; o[it][2][q] = s2; o[it][3][q] = s3; o[it][4][q] = s4;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < HIT; ++it) {
    const int e = tid + it * 256;
    if (e >= HT) break;
    const int r = e >> 4, c0 = (e & 15) * 4;
#pragma unroll
    for (int m = 0; m < 5; ++m)
      *reinterpret_cast<float4*>(&hm[m][r][c0]) = make_float4(o[it][m][0], o[it][m][1], o[it][m][2], o[it][m][3]);
  }
  __syncthreads();
  // vertical pass + SSIM map: one column, four consecutive output rows per task
  double sacc = 0.0;
  for (int e = tid; e < (SS_TH / 4) * SS_TW; e += 256) {
    const int r0 = (e / SS_TW) * 4, c = e % SS_TW;
    const int gx = x0 + c;
    if (gx >= W || y0 + r0 >= H) continue;
    float h[5][14];
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int i = 0; i < 14; ++i) h[m][i] = hm[m][r0 + i][c];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int gy = y0 + r0 + q;
      if (gy >= H) break;
      float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const float k = win.k[t];
#pragma unroll
        for (int m = 0; m < 5; ++m) v[m] = fmaf(k, h[m][q + t], v[m]);
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
      const long o = (plane * H + gy) * W + gx;
      if (lmap) lmap[o] = lc;
      if (coef) {
        const float dS = (l >= 0.f && l <= 1.f) ? -0.5f * inv_n : 0.f;
        // dnum/dmx = 2 my (A2 - A1); dden/dmx = 2 mx (B2 - B1); dS/dE[x^2] = -S B1 / D; dS/dE[xy] = 2 A1 / D
        const float dmx = (2.f * my * (A2 - A1) - S * 2.f * mx * (B2 - B1)) / D;
        const float dxx = -S * B1 / D;
        const float dxy = 2.f * A1 / D;
        coef[o] = dS * dmx;
        coef[n + o] = dS * dxx;
        coef[2 * n + o] = dS * dxy;
      }
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
// rows [n-5, n) with j >= y0.  Interior groups of 4 rows (columns) run register-blocked; a group touching the
// reflected border runs the per-output gather.
constexpr int SB_TH = 16, SB_TW = 64, SB_M = 5;
constexpr int SB_P = SB_TW + 2 * SB_M + 2;

__device__ __forceinline__ int refl_sources(int j, int n, int* qs) {
  int nq = 0;
  qs[nq++] = j;
  if (j >= 1 && j <= 5) qs[nq++] = -j;
  if (j <= n - 2 && j >= n - 6) qs[nq++] = 2 * (n - 1) - j;
  return nq;
}

// The reflected sources' taps of output j (after its direct window, in refl_sources order): only the lanes of the
// five outputs next to each border run any; the direct window itself is the interior formula, the staged values
// outside the image being zero.  lo: the source position of LDS index 0; NP: the LDS stride of one position; MS: of
// one map.
template <int NP, int MS>
__device__ __forceinline__ void refl_extra(int j, int n, int lo, const Win& win, const float* __restrict__ base,
                                           float& a0, float& a1, float& a2) {
  int qs[3];
  const int nq = refl_sources(j, n, qs);
  for (int u = 1; u < nq; ++u) {
    for (int t = 0; t < 11; ++t) {
      const int rr = qs[u] - t + 5;
      if (rr < 0 || rr >= n) continue;
      const int l = (rr - lo) * NP;
      const float k = win.k[t];
      a0 = fmaf(k, base[l], a0);
      a1 = fmaf(k, base[l + MS], a1);
      a2 = fmaf(k, base[l + 2 * MS], a2);
    }
  }
}

// up_map (optional, reduction 'none'): the per-pixel upstream gradient, applied to the coefficients as they are
// staged (the adjoint filters are linear); otherwise the scalar up[0] scales the result
__global__ __launch_bounds__(256) void ssim_bwd_tiled(const float* __restrict__ coef, const float* __restrict__ x,
                                                       const float* __restrict__ y, int H, int W, Win win,
                                                       int clamp_in, const float* __restrict__ up,
                                                       const float* __restrict__ up_map, float* __restrict__ gx,
                                                       long n) {
  constexpr int LH = SB_TH + 2 * SB_M, LW = SB_TW + 2 * SB_M;
  // tv (the vertical adjoint) overwrites cs once every task holds its outputs in registers: 24 KB of LDS per 16-row
  // tile, six tiles per CU (16-row tiles: 52.5 -> 40.2 us at cfg2 against 32-row ones, whose 1.5 rounds of 4 tiles per
  // CU left half the chip idle in the second)
  __shared__ __attribute__((aligned(16))) float sbuf[3 * LH * SB_P];
  auto cs = reinterpret_cast<float (*)[LH][SB_P]>(sbuf);
  auto tv = reinterpret_cast<float (*)[SB_TH][SB_P]>(sbuf);
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * SB_TW, y0 = blockIdx.y * SB_TH;
  const long plane = blockIdx.z;
  const long pb = plane * H * W;
  // every coefficient load of the thread's NB positions issued before the first LDS store
  constexpr int NB = (LH * LW + 255) / 256;
  float v[NB][3];
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int e = tid + u * 256;
    const int r = e / LW, c = e % LW;
    const int gy = y0 - SB_M + r, gxx = x0 - SB_M + c;
    const bool in = e < LH * LW && gy >= 0 && gy < H && gxx >= 0 && gxx < W;
    const long o = pb + (long)gy * W + gxx;
    const float um = in && up_map ? up_map[o] : 1.f;
#pragma unroll
    for (int m = 0; m < 3; ++m) v[u][m] = in ? coef[m * n + o] * um : 0.f;
  }
#pragma unroll
  for (int u = 0; u < NB; ++u) {
    const int e = tid + u * 256;
    if (e >= LH * LW) break;
    const int r = e / LW, c = e % LW;
#pragma unroll
    for (int m = 0; m < 3; ++m) cs[m][r][c] = v[u][m];
  }
  // this thread's output pixels of x / y (two tasks of one row x four columns), loaded now so their latency overlaps
  // the two adjoint passes
  constexpr int PER = SB_TH * SB_TW / (4 * 256);
  // float4 paths only for 16-byte aligned rows: W a multiple of 4 AND 16-byte aligned bases (a public C-ABI entry may
  // receive a view with an odd element offset)
  const bool vec = (W & 3) == 0 && (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gx) & 15) == 0;
  float xo[PER][4], yo[PER][4];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + k * 256, r = e >> 4, c0 = (e & 15) * 4;
    const int j = y0 + r, i0 = x0 + c0;
    const long o = pb + (long)j * W + i0;
    if (j < H && vec && i0 + 3 < W) {
      const float4 a = *reinterpret_cast<const float4*>(x + o);
      const float4 b = *reinterpret_cast<const float4*>(y + o);
      xo[k][0] = a.x; xo[k][1] = a.y; xo[k][2] = a.z; xo[k][3] = a.w;
      yo[k][0] = b.x; yo[k][1] = b.y; yo[k][2] = b.z; yo[k][3] = b.w;
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = j < H && i0 + q < W;
        xo[k][q] = ok ? x[o + q] : 0.f;
        yo[k][q] = ok ? y[o + q] : 0.f;
      }
    }
  }
  __syncthreads();
  // vertical adjoint for the tile's rows and every staged column: one column, four consecutive rows per task
  constexpr int VT = (SB_TH / 4) * LW, VIT = (VT + 255) / 256;
  float tvo[VIT][3][4];
#pragma unroll
  for (int it = 0; it < VIT; ++it) {
    const int e = tid + it * 256;
    if (e >= VT) break;
    const int r0 = (e / LW) * 4, c = e % LW;
    const int j0 = y0 + r0;
    float w[3][14];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int i = 0; i < 14; ++i) w[m][i] = cs[m][r0 + i][c];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float a[3] = {0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const float k = win.k[t];
#pragma unroll
        for (int m = 0; m < 3; ++m) a[m] = fmaf(k, w[m][q + 10 - t], a[m]);
      }
      const int j = j0 + q;
      if ((j < 6 || j > H - 7) && j < H)
        refl_extra<SB_P, LH * SB_P>(j, H, y0 - SB_M, win, &cs[0][0][c], a[0], a[1], a[2]);
#pragma unroll
      for (int m = 0; m < 3; ++m) tvo[it][m][q] = a[m];
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < VIT; ++it) {
    const int e = tid + it * 256;
    if (e >= VT) break;
    const int r0 = (e / LW) * 4, c = e % LW;
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) tv[m][r0 + q][c] = tvo[it][m][q];
  }
  __syncthreads();
  const float g0 = up_map ? 1.f : up[0];
  // horizontal adjoint + the pixel gradient: one row, four consecutive columns per task
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + k * 256, r = e >> 4, c0 = (e & 15) * 4;
    const int j = y0 + r, i0 = x0 + c0;
    if (j >= H || i0 >= W) continue;
    float w[3][16];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const float4 f = *reinterpret_cast<const float4*>(&tv[m][r][c0 + 4 * s4]);
        w[m][4 * s4] = f.x; w[m][4 * s4 + 1] = f.y; w[m][4 * s4 + 2] = f.z; w[m][4 * s4 + 3] = f.w;
      }
    float a[3][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[0][q] = a[1][q] = a[2][q] = 0.f;
#pragma unroll
      for (int t = 0; t < 11; ++t) {
        const float kk = win.k[t];
#pragma unroll
        for (int m = 0; m < 3; ++m) a[m][q] = fmaf(kk, w[m][q + 10 - t], a[m][q]);
      }
      const int i = i0 + q;
      if ((i < 6 || i > W - 7) && i < W) refl_extra<1, SB_TH * SB_P>(i, W, x0 - SB_M, win, &tv[0][r][0], a[0][q], a[1][q], a[2][q]);
    }
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float xr = xo[k][q];
      float xv = xr, yv = yo[k][q];
      if (clamp_in) { xv = clamp01(xv); yv = clamp01(yv); }
      float gq = a[0][q] + 2.f * xv * a[1][q] + yv * a[2][q];
      if (clamp_in && !(xr >= 0.f && xr <= 1.f)) gq = 0.f;
      g[q] = g0 * gq;
    }
    const long o = pb + (long)j * W + i0;
    if (vec && i0 + 3 < W) {
      *reinterpret_cast<float4*>(gx + o) = make_float4(g[0], g[1], g[2], g[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (i0 + q < W) gx[o + q] = g[q];
    }
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
  NBP_REQUIRE((reduction == 2 ? lmap != nullptr : loss != nullptr) || (want_grad && !loss && !lmap),
              "nbp_ssim_loss_fwd: output missing for the reduction");
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
