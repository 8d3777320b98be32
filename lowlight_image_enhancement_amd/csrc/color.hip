// Colour-difference kernels on NCHW sRGB [B][3][H][W] fp32:
//   * the DeltaE00 LOSS form (NewBP_model/losses.py:92-143): kornia-0.6.12 rgb_to_lab (restated, oracle/losses.py)
//     of clamp01 inputs, the reference's non-standard _ciede2000 (eps 1e-6, h wrapped mod 2pi, R_T = -sin(rad(dro)) R_C),
//     mean over pixels; forward and d/d(gen);
//   * the DeltaE00 METRIC map (metrics/color_error.py:105-210, deltaE2000_map :235-267): unwrapped hue, c1'c2'==0
//     special cases, R_T = -sin(2 dtheta) R_C, /(k S + eps), sqrt(clamp >= 0).
// The loss gradient is forward-mode AD: every quantity is a dual number carrying d/d(R,G,B) of the generated pixel,
// so branch selectors (where / comparisons / the mod-2pi wrap / clamp masks) take autograd's semantics exactly and
// one pass gives dE and its three partials.  All arithmetic fp32 with the reference's fp32 constants.
#include "nbp_common.h"

using namespace nbp;

namespace {

struct D3 {
  float v, d0, d1, d2;
};
__device__ __forceinline__ D3 mk(float v) { return D3{v, 0.f, 0.f, 0.f}; }
__device__ __forceinline__ D3 scl(const D3& a, float dv, float vv) { return D3{vv, a.d0 * dv, a.d1 * dv, a.d2 * dv}; }
__device__ __forceinline__ D3 operator+(const D3& a, const D3& b) { return D3{a.v + b.v, a.d0 + b.d0, a.d1 + b.d1, a.d2 + b.d2}; }
__device__ __forceinline__ D3 operator-(const D3& a, const D3& b) { return D3{a.v - b.v, a.d0 - b.d0, a.d1 - b.d1, a.d2 - b.d2}; }
__device__ __forceinline__ D3 operator*(const D3& a, const D3& b) {
  return D3{a.v * b.v, a.d0 * b.v + a.v * b.d0, a.d1 * b.v + a.v * b.d1, a.d2 * b.v + a.v * b.d2};
}
__device__ __forceinline__ D3 operator/(const D3& a, const D3& b) {
  const float q = a.v / b.v, ib = 1.f / b.v;
  return D3{q, (a.d0 - q * b.d0) * ib, (a.d1 - q * b.d1) * ib, (a.d2 - q * b.d2) * ib};
}
__device__ __forceinline__ D3 operator+(const D3& a, float b) { return D3{a.v + b, a.d0, a.d1, a.d2}; }
__device__ __forceinline__ D3 operator+(float b, const D3& a) { return a + b; }
__device__ __forceinline__ D3 operator-(const D3& a, float b) { return D3{a.v - b, a.d0, a.d1, a.d2}; }
__device__ __forceinline__ D3 operator-(float b, const D3& a) { return D3{b - a.v, -a.d0, -a.d1, -a.d2}; }
__device__ __forceinline__ D3 operator-(const D3& a) { return D3{-a.v, -a.d0, -a.d1, -a.d2}; }
__device__ __forceinline__ D3 operator*(const D3& a, float b) { return D3{a.v * b, a.d0 * b, a.d1 * b, a.d2 * b}; }
__device__ __forceinline__ D3 operator*(float b, const D3& a) { return a * b; }
__device__ __forceinline__ D3 operator/(const D3& a, float b) { return D3{a.v / b, a.d0 / b, a.d1 / b, a.d2 / b}; }

__device__ __forceinline__ float val(float x) { return x; }
__device__ __forceinline__ float val(const D3& x) { return x.v; }

__device__ __forceinline__ float vsqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ D3 vsqrt(const D3& x) {
  const float r = sqrtf(x.v);
  return scl(x, 0.5f / r, r);
}
__device__ __forceinline__ float vpow(float x, float c) { return powf(x, c); }
__device__ __forceinline__ D3 vpow(const D3& x, float c) { return scl(x, c * powf(x.v, c - 1.f), powf(x.v, c)); }
__device__ __forceinline__ float vsin(float x) { return sinf(x); }
__device__ __forceinline__ D3 vsin(const D3& x) { return scl(x, cosf(x.v), sinf(x.v)); }
__device__ __forceinline__ float vcos(float x) { return cosf(x); }
__device__ __forceinline__ D3 vcos(const D3& x) { return scl(x, -sinf(x.v), cosf(x.v)); }
__device__ __forceinline__ float vexp(float x) { return expf(x); }
__device__ __forceinline__ D3 vexp(const D3& x) {
  const float e = expf(x.v);
  return scl(x, e, e);
}
__device__ __forceinline__ float vatan2(float y, float x) { return atan2f(y, x); }
// torch's atan2 backward is defined as 0 at the origin (a grey pixel: a' = b = 0)
__device__ __forceinline__ D3 vatan2(const D3& y, const D3& x) {
  const float den = x.v * x.v + y.v * y.v, v = atan2f(y.v, x.v);
  if (den == 0.f) return mk(v);
  return D3{v, (x.v * y.d0 - y.v * x.d0) / den, (x.v * y.d1 - y.v * x.d1) / den, (x.v * y.d2 - y.v * x.d2) / den};
}
// torch remainder (sign of the divisor): a - b * floor(a / b); d/da = 1
__device__ __forceinline__ float vmod(float a, float b) { return a - b * floorf(a / b); }
__device__ __forceinline__ D3 vmod(const D3& a, float b) { return D3{vmod(a.v, b), a.d0, a.d1, a.d2}; }
// clamp(min=lo): identity slope where x >= lo (torch's inclusive mask), constant below
__device__ __forceinline__ float vclamp_min(float x, float lo) { return fmaxf(x, lo); }
__device__ __forceinline__ D3 vclamp_min(const D3& x, float lo) { return x.v >= lo ? x : mk(lo); }
template <typename V>
__device__ __forceinline__ V sel(bool c, const V& a, const V& b) { return c ? a : b; }

constexpr float PI_F = 3.14159265358979323846f;
constexpr float TWO_PI_F = 6.28318530717958647692f;
constexpr float P25 = 6103515625.f;  // 25**7 as the fp32 scalar torch adds
constexpr float DEG2RAD = 0.017453292519943295f, RAD2DEG = 57.29577951308232f;

// kornia 0.6.12 color.rgb_to_lab for one pixel (inputs already clamped as the caller requires)
template <typename V>
__device__ __forceinline__ void rgb_to_lab(const V& r0, const V& g0, const V& b0, V& L, V& A, V& Bc) {
  auto lin = [](const V& x) { return sel(val(x) > 0.04045f, vpow((x + 0.055f) / 1.055f, 2.4f), x / 12.92f); };
  const V r = lin(r0), g = lin(g0), b = lin(b0);
  const V X = 0.412453f * r + 0.357580f * g + 0.180423f * b;
  const V Y = 0.212671f * r + 0.715160f * g + 0.072169f * b;
  const V Z = 0.019334f * r + 0.119193f * g + 0.950227f * b;
  auto f = [](const V& t) {
    const float thr = 0.008856f;
    return sel(val(t) > thr, vpow(vclamp_min(t, thr), 1.f / 3.f), 7.787f * t + 4.f / 29.f);
  };
  const V fx = f(X / 0.95047f), fy = f(Y / 1.f), fz = f(Z / 1.08883f);
  L = 116.f * fy - 16.f;
  A = 500.f * (fx - fy);
  Bc = 200.f * (fy - fz);
}

// DeltaE00Loss._ciede2000 (losses.py:98-136), per pixel
template <typename V>
__device__ __forceinline__ V ciede2000_loss(const V& L1, const V& a1, const V& b1, const V& L2, const V& a2, const V& b2,
                                            float eps) {
  const V C1 = vsqrt(a1 * a1 + b1 * b1 + eps);
  const V C2 = vsqrt(a2 * a2 + b2 * b2 + eps);
  const V Cb = 0.5f * (C1 + C2);
  const V Cb7 = vpow(Cb, 7.f);
  const V G = 0.5f * (1.f - vsqrt(Cb7 / ((Cb7 + P25) + eps)));
  const V a1p = (1.f + G) * a1, a2p = (1.f + G) * a2;
  const V C1p = vsqrt(a1p * a1p + b1 * b1 + eps);
  const V C2p = vsqrt(a2p * a2p + b2 * b2 + eps);
  const V h1p = vmod(vatan2(b1, a1p), TWO_PI_F);
  const V h2p = vmod(vatan2(b2, a2p), TWO_PI_F);
  const V dLp = L2 - L1;
  const V dCp = C2p - C1p;
  V dhp = h2p - h1p;
  dhp = dhp - TWO_PI_F * (float)(val(dhp) > PI_F) + TWO_PI_F * (float)(val(dhp) < -PI_F);
  const V dHp = 2.f * vsqrt(C1p * C2p + eps) * vsin(dhp / 2.f);
  const V Lb = 0.5f * (L1 + L2);
  const V Cbp = 0.5f * (C1p + C2p);
  const V hs = h1p + h2p;
  const V hbp = hs / 2.f - PI_F * (float)(fabsf(val(h1p) - val(h2p)) > PI_F) + TWO_PI_F * (float)(val(hs) < 0.f);
  const float d30 = 30.f * DEG2RAD, d6 = 6.f * DEG2RAD, d63 = 63.f * DEG2RAD;
  const V T = 1.f - 0.17f * vcos(hbp - d30) + 0.24f * vcos(2.f * hbp) + 0.32f * vcos(3.f * hbp + d6) -
              0.20f * vcos(4.f * hbp - d63);
  const V u = (hbp * RAD2DEG - 275.f) / 25.f;
  const V dro = 30.f * vexp(-(u * u));
  const V Cbp7 = vpow(Cbp, 7.f);
  const V RC = 2.f * vsqrt(Cbp7 / ((Cbp7 + P25) + eps));
  const V l50 = Lb - 50.f;
  const V SL = 1.f + (0.015f * (l50 * l50)) / vsqrt(20.f + l50 * l50 + eps);
  const V SC = 1.f + 0.045f * Cbp;
  const V SH = 1.f + 0.015f * Cbp * T;
  const V RT = -vsin(dro * DEG2RAD) * RC;
  const V tL = dLp / SL, tC = dCp / SC, tH = dHp / SH;
  return vsqrt(tL * tL + tC * tC + tH * tH + RT * tC * tH + eps);
}

// _deltaE00_lab_map (color_error.py:105-210), per pixel (no gradient: a no-grad metric)
__device__ __forceinline__ float ciede2000_metric(float L1, float a1, float b1, float L2, float a2, float b2, float kL,
                                                  float kC, float kH, float eps) {
  const float c1 = sqrtf(a1 * a1 + b1 * b1 + eps), c2 = sqrtf(a2 * a2 + b2 * b2 + eps);
  const float cb7 = powf(0.5f * (c1 + c2), 7.f);
  const float g = 0.5f * (1.f - sqrtf(cb7 / (cb7 + P25 + eps)));
  const float a1p = (1.f + g) * a1, a2p = (1.f + g) * a2;
  const float c1p = sqrtf(a1p * a1p + b1 * b1 + eps), c2p = sqrtf(a2p * a2p + b2 * b2 + eps);
  const float h1p = atan2f(b1, a1p), h2p = atan2f(b2, a2p);
  const float dLp = L2 - L1, dCp = c2p - c1p;
  const bool valid = (c1p * c2p) != 0.f;
  const float diff = h2p - h1p;
  float dh = 0.f;
  if (valid) {
    if (fabsf(diff) <= PI_F) dh = diff;
    else if (diff > PI_F) dh = diff - 2.f * PI_F;
    else dh = diff + 2.f * PI_F;
  }
  const float dHp = 2.f * sqrtf(c1p * c2p + eps) * sinf(dh / 2.f);
  const float Lbp = 0.5f * (L1 + L2), Cbp = 0.5f * (c1p + c2p);
  const float hs = h1p + h2p, ad = fabsf(h1p - h2p);
  const float hb = !valid ? hs : (ad <= PI_F ? 0.5f * hs : (hs < 2.f * PI_F ? 0.5f * (hs + 2.f * PI_F) : 0.5f * (hs - 2.f * PI_F)));
  const float r30 = 30.f * PI_F / 180.f, r6 = 6.f * PI_F / 180.f, r63 = 63.f * PI_F / 180.f;
  const float T = 1.f - 0.17f * cosf(hb - r30) + 0.24f * cosf(2.f * hb) + 0.32f * cosf(3.f * hb + r6) -
                  0.20f * cosf(4.f * hb - r63);
  const float u = ((hb * 180.f / PI_F) - 275.f) / 25.f;
  const float dtheta = r30 * expf(-(u * u));
  const float cbp7 = powf(Cbp, 7.f);
  const float RC = 2.f * sqrtf(cbp7 / (cbp7 + P25 + eps));
  const float RT = -sinf(2.f * dtheta) * RC;
  const float l50 = Lbp - 50.f;
  const float SL = 1.f + (0.015f * l50 * l50) / sqrtf(20.f + l50 * l50 + eps);
  const float SC = 1.f + 0.045f * Cbp, SH = 1.f + 0.015f * Cbp * T;
  const float tL = dLp / (kL * SL + eps), tC = dCp / (kC * SC + eps), tH = dHp / (kH * SH + eps);
  return sqrtf(fmaxf(tL * tL + tC * tC + tH * tH + RT * tC * tH, 0.f));
}

__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }

__global__ __launch_bounds__(256) void de00_loss_fwd_kernel(const float* __restrict__ gen, const float* __restrict__ tgt,
                                                            long HW, long npix, int clamp, float eps,
                                                            double* __restrict__ part) {
  __shared__ double red[16];
  double acc = 0.0;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const long o = b * 3 * HW + q;
    float r1 = gen[o], g1 = gen[o + HW], b1 = gen[o + 2 * HW];
    float r2 = tgt[o], g2 = tgt[o + HW], b2 = tgt[o + 2 * HW];
    if (clamp) {
      r1 = clamp01(r1); g1 = clamp01(g1); b1 = clamp01(b1);
      r2 = clamp01(r2); g2 = clamp01(g2); b2 = clamp01(b2);
    }
    float L1, A1, B1, L2, A2, B2;
    rgb_to_lab(r1, g1, b1, L1, A1, B1);
    rgb_to_lab(r2, g2, b2, L2, A2, B2);
    acc += (double)ciede2000_loss(L1, A1, B1, L2, A2, B2, eps);
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void de00_finalize(const double* __restrict__ part, int n, double inv, float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += part[i];
    out[0] = (float)(s * inv);
  }
}

// dgen = up[0] / npix * d dE / d gen  (through clamp01's inclusive mask when clamp != 0)
__global__ __launch_bounds__(256) void de00_loss_bwd_kernel(const float* __restrict__ gen, const float* __restrict__ tgt,
                                                            long HW, long npix, int clamp, float eps,
                                                            const float* __restrict__ up, float* __restrict__ dgen) {
  const float scale = up[0] / (float)npix;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const long o = b * 3 * HW + q;
    const float x0 = gen[o], x1 = gen[o + HW], x2 = gen[o + 2 * HW];
    float r2 = tgt[o], g2 = tgt[o + HW], b2 = tgt[o + 2 * HW];
    if (clamp) {
      r2 = clamp01(r2); g2 = clamp01(g2); b2 = clamp01(b2);
    }
    const float m0 = !clamp || (x0 >= 0.f && x0 <= 1.f) ? 1.f : 0.f;
    const float m1 = !clamp || (x1 >= 0.f && x1 <= 1.f) ? 1.f : 0.f;
    const float m2 = !clamp || (x2 >= 0.f && x2 <= 1.f) ? 1.f : 0.f;
    const D3 R{clamp ? clamp01(x0) : x0, m0, 0.f, 0.f};
    const D3 G{clamp ? clamp01(x1) : x1, 0.f, m1, 0.f};
    const D3 Bb{clamp ? clamp01(x2) : x2, 0.f, 0.f, m2};
    D3 L1, A1, B1;
    rgb_to_lab(R, G, Bb, L1, A1, B1);
    float L2, A2, B2;
    rgb_to_lab(r2, g2, b2, L2, A2, B2);
    const D3 dE = ciede2000_loss(L1, A1, B1, mk(L2), mk(A2), mk(B2), eps);
    dgen[o] = scale * dE.d0;
    dgen[o + HW] = scale * dE.d1;
    dgen[o + 2 * HW] = scale * dE.d2;
  }
}

__global__ __launch_bounds__(256) void de00_metric_kernel(const float* __restrict__ pred, const float* __restrict__ tgt,
                                                          long HW, long npix, float kL, float kC, float kH, float eps,
                                                          float* __restrict__ map) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const long o = b * 3 * HW + q;
    float L1, A1, B1, L2, A2, B2;
    rgb_to_lab(pred[o], pred[o + HW], pred[o + 2 * HW], L1, A1, B1);
    rgb_to_lab(tgt[o], tgt[o + HW], tgt[o + 2 * HW], L2, A2, B2);
    map[p] = ciede2000_metric(L1, A1, B1, L2, A2, B2, kL, kC, kH, eps);
  }
}

// both CIEDE2000 forms on Lab inputs [B][3][H][W] (pins the formulas against the Sharma pairs without rgb_to_lab)
__global__ __launch_bounds__(256) void de00_lab_kernel(const float* __restrict__ lab1, const float* __restrict__ lab2,
                                                       long HW, long npix, int form, float kL, float kC, float kH,
                                                       float eps, float* __restrict__ out) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const long o = b * 3 * HW + q;
    const float L1 = lab1[o], A1 = lab1[o + HW], B1 = lab1[o + 2 * HW];
    const float L2 = lab2[o], A2 = lab2[o + HW], B2 = lab2[o + 2 * HW];
    out[p] = form == 0 ? ciede2000_loss(L1, A1, B1, L2, A2, B2, eps)
                       : ciede2000_metric(L1, A1, B1, L2, A2, B2, kL, kC, kH, eps);
  }
}

// d/d lab1 of the loss-form CIEDE2000 on Lab inputs (DeltaE00Loss._ciede2000's autograd, losses.py:98-136): dual
// numbers carry d/d(L1, a1, b1); d1 = g[p] * partials.  The formula is symmetric in its two arguments (every
// difference enters squared or as the product dC' dH'), so the caller gets d/d lab2 by swapping the inputs.
__global__ __launch_bounds__(256) void de00_lab_bwd_kernel(const float* __restrict__ lab1, const float* __restrict__ lab2,
                                                           long HW, long npix, float eps, const float* __restrict__ g,
                                                           float* __restrict__ d1) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const long o = b * 3 * HW + q;
    const D3 L1{lab1[o], 1.f, 0.f, 0.f}, A1{lab1[o + HW], 0.f, 1.f, 0.f}, B1{lab1[o + 2 * HW], 0.f, 0.f, 1.f};
    const D3 dE = ciede2000_loss(L1, A1, B1, mk(lab2[o]), mk(lab2[o + HW]), mk(lab2[o + 2 * HW]), eps);
    const float gp = g[p];
    d1[o] = gp * dE.d0;
    d1[o + HW] = gp * dE.d1;
    d1[o + 2 * HW] = gp * dE.d2;
  }
}

// Lab of NCHW sRGB (kornia rgb_to_lab), for callers that need the L channel (edge_deltaE2000)
__global__ __launch_bounds__(256) void rgb_to_lab_kernel(const float* __restrict__ rgb, long HW, long npix,
                                                         float* __restrict__ lab) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < npix; p += (long)gridDim.x * blockDim.x) {
    const long b = p / HW, q = p - b * HW;
    const long o = b * 3 * HW + q;
    float L, A, Bc;
    rgb_to_lab(rgb[o], rgb[o + HW], rgb[o + 2 * HW], L, A, Bc);
    lab[o] = L;
    lab[o + HW] = A;
    lab[o + 2 * HW] = Bc;
  }
}

inline int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 2048 ? 2048 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

size_t nbp_de00_workspace_doubles(long npix) { return (size_t)grid_for(npix); }

int nbp_de00_loss_fwd(const float* gen, const float* tgt, int B, int H, int W, int clamp, float eps, double* ws,
                      float* out, nbp_stream_t s) {
  NBP_REQUIRE(gen && tgt && ws && out && B > 0 && H > 0 && W > 0, "nbp_de00_loss_fwd: bad args");
  const long HW = (long)H * W, npix = B * HW;
  const int g = grid_for(npix);
  de00_loss_fwd_kernel<<<g, 256, 0, S(s)>>>(gen, tgt, HW, npix, clamp, eps, ws);
  de00_finalize<<<1, 64, 0, S(s)>>>(ws, g, 1.0 / (double)npix, out);
  return check_launch("de00_loss_fwd");
}

int nbp_de00_loss_bwd(const float* gen, const float* tgt, int B, int H, int W, int clamp, float eps, const float* up,
                      float* dgen, nbp_stream_t s) {
  NBP_REQUIRE(gen && tgt && up && dgen && B > 0 && H > 0 && W > 0, "nbp_de00_loss_bwd: bad args");
  const long HW = (long)H * W, npix = B * HW;
  de00_loss_bwd_kernel<<<grid_for(npix), 256, 0, S(s)>>>(gen, tgt, HW, npix, clamp, eps, up, dgen);
  return check_launch("de00_loss_bwd");
}

int nbp_de00_metric_map(const float* pred, const float* tgt, int B, int H, int W, float kL, float kC, float kH,
                        float eps, float* map, nbp_stream_t s) {
  NBP_REQUIRE(pred && tgt && map && B > 0 && H > 0 && W > 0 && eps > 0.f, "nbp_de00_metric_map: bad args");
  const long HW = (long)H * W, npix = B * HW;
  de00_metric_kernel<<<grid_for(npix), 256, 0, S(s)>>>(pred, tgt, HW, npix, kL, kC, kH, eps, map);
  return check_launch("de00_metric_map");
}

int nbp_de00_lab(const float* lab1, const float* lab2, int B, int H, int W, int form, float kL, float kC, float kH,
                 float eps, float* out, nbp_stream_t s) {
  NBP_REQUIRE(lab1 && lab2 && out && B > 0 && H > 0 && W > 0 && (form == 0 || form == 1), "nbp_de00_lab: bad args");
  const long HW = (long)H * W, npix = B * HW;
  de00_lab_kernel<<<grid_for(npix), 256, 0, S(s)>>>(lab1, lab2, HW, npix, form, kL, kC, kH, eps, out);
  return check_launch("de00_lab");
}

int nbp_de00_lab_bwd(const float* lab1, const float* lab2, int B, int H, int W, float eps, const float* g, float* d1,
                     nbp_stream_t s) {
  NBP_REQUIRE(lab1 && lab2 && g && d1 && B > 0 && H > 0 && W > 0, "nbp_de00_lab_bwd: bad args");
  const long HW = (long)H * W, npix = B * HW;
  de00_lab_bwd_kernel<<<grid_for(npix), 256, 0, S(s)>>>(lab1, lab2, HW, npix, eps, g, d1);
  return check_launch("de00_lab_bwd");
}

int nbp_rgb_to_lab(const float* rgb, int B, int H, int W, float* lab, nbp_stream_t s) {
  NBP_REQUIRE(rgb && lab && B > 0 && H > 0 && W > 0, "nbp_rgb_to_lab: bad args");
  const long HW = (long)H * W, npix = B * HW;
  rgb_to_lab_kernel<<<grid_for(npix), 256, 0, S(s)>>>(rgb, HW, npix, lab);
  return check_launch("rgb_to_lab");
}

}  // extern "C"
