// NAFBlock spatial branch on NHWC activations (NAFNet_arch.py:32-41,64-67):
//   conv2 = depthwise 3x3 (zero pad 1, bias) on 2C channels  ->  SimpleGate (x[:C] * x[C:])
//   -> SCA: AdaptiveAvgPool2d(1) -> 1x1 conv C->C (+bias) -> broadcast multiply.
// The pool is a per-image global reduction: the forward writes per-(image, chunk) partial sums in a slab that the
// SCA kernel folds in a fixed order (bitwise reproducible, no atomics).
#include "nbp_common.h"
#include "sca_bwd.h"

using namespace nbp;

namespace {

struct Geo {
  int B, H, W, C;  // C = gate width; the depthwise conv runs on 2C channels
  int chunks;      // pixel chunks per image
  int chunk_px;    // pixels per chunk
};

// thread layout: quad q (4 channels) = tid % Q, pixel lane = tid / Q, PPI = blockDim / Q pixels per step
template <typename T>
__global__ void dw_sg_pool_fwd(const T* __restrict__ t1, const float* __restrict__ wdw, const float* __restrict__ bdw,
                               T* __restrict__ t2, T* __restrict__ g, float* __restrict__ pool_slab, Geo geo) {
  extern __shared__ float red[];  // [blockDim][4]
  const int C = geo.C, C2 = 2 * C, Q = C / 4;
  const int tid = threadIdx.x, q = tid % Q, pl = tid / Q, PPI = blockDim.x / Q;
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int HW = geo.H * geo.W;
  float wa[4][9], wb[4][9];
  float4 ba = ld4(bdw + q * 4), bb = ld4(bdw + C + q * 4);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      wa[j][t] = wdw[(q * 4 + j) * 9 + t];
      wb[j][t] = wdw[(C + q * 4 + j) * 9 + t];
    }
  float4 pacc = f4(0.f);
  const int p0 = chunk * geo.chunk_px, p1 = min(HW, p0 + geo.chunk_px);
  const T* base = t1 + (long)b * HW * C2;
  if (pl < PPI) {
    for (int p = p0 + pl; p < p1; p += PPI) {
      const int h = p / geo.W, w = p - h * geo.W;
      float4 aa = ba, ab = bb;
#pragma unroll
      for (int dh = -1; dh <= 1; ++dh) {
        const int hh = h + dh;
        if (hh < 0 || hh >= geo.H) continue;
#pragma unroll
        for (int dw = -1; dw <= 1; ++dw) {
          const int ww = w + dw;
          if (ww < 0 || ww >= geo.W) continue;
          const int t = (dh + 1) * 3 + (dw + 1);
          const T* src = base + ((long)hh * geo.W + ww) * C2 + q * 4;
          const float4 va = ldq(src), vb = ldq(src + C);
          aa.x = fmaf(wa[0][t], va.x, aa.x); aa.y = fmaf(wa[1][t], va.y, aa.y);
          aa.z = fmaf(wa[2][t], va.z, aa.z); aa.w = fmaf(wa[3][t], va.w, aa.w);
          ab.x = fmaf(wb[0][t], vb.x, ab.x); ab.y = fmaf(wb[1][t], vb.y, ab.y);
          ab.z = fmaf(wb[2][t], vb.z, ab.z); ab.w = fmaf(wb[3][t], vb.w, ab.w);
        }
      }
      const long m = (long)b * HW + p;
      stq(t2 + m * C2 + q * 4, aa);
      stq(t2 + m * C2 + C + q * 4, ab);
      const float4 gv = aa * ab;
      stq(g + m * C + q * 4, gv);
      pacc += gv;
    }
  }
  st4(red + tid * 4, pacc);
  __syncthreads();
  if (pl == 0) {
    float4 s = f4(0.f);
    for (int k = 0; k < PPI; ++k) s += ld4(red + (k * Q + q) * 4);
    st4(pool_slab + ((long)b * geo.chunks + chunk) * C + q * 4, s);
  }
}

// out[b][c] = scale * sum_{k < chunks} slab[b][k][c]: 8 lanes per element, lane j sums chunks k = j (mod 8) with
// independent loads, then a fixed-order xor combine (deterministic).  Feeds the SCA GEMVs with finished vectors.
__global__ __launch_bounds__(256) void reduce_rows8(const float* __restrict__ slab, int B, int chunks, int C,
                                                    float scale, float* __restrict__ out) {
  const int e = blockIdx.x * 32 + (threadIdx.x >> 3), j = threadIdx.x & 7;
  float acc = 0.f;
  if (e < B * C) {
    const int b = e / C, c = e - b * C;
    const float* src = slab + (long)b * chunks * C + c;
    float a0 = 0.f, a1 = 0.f;
    int k = j;
    for (; k + 8 < chunks; k += 16) {
      a0 += src[(long)k * C];
      a1 += src[(long)(k + 8) * C];
    }
    if (k < chunks) a0 += src[(long)k * C];
    acc = a0 + a1;
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (j == 0 && e < B * C) out[e] = acc * scale;
}

// images per block of the unfused SCA backward (sca_bwd_ds)
constexpr int SCA_NB = 16;

// sum_{k < chunks} slab[b][k][c] with 4 independent accumulators, fixed order (the pooled / reduced vector element)
__device__ __forceinline__ float chunk_sum(const float* __restrict__ slab, int chunks, int C, int b, int c) {
  const float* src = slab + (long)b * chunks * C + c;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int k = 0;
  for (; k + 3 < chunks; k += 4) {
    a0 += src[(long)k * C];
    a1 += src[(long)(k + 1) * C];
    a2 += src[(long)(k + 2) * C];
    a3 += src[(long)(k + 3) * C];
  }
  for (; k < chunks; ++k) a0 += src[(long)k * C];
  return (a0 + a1) + (a2 + a3);
}

// Stage sm[e] = scale * sum_{k < chunks} slab[b0 + e / CW][k][c0 + e % CW] for e < nE with the loads batched (16 in flight
// per thread: 4 elements x 4 chunks).  When the block has more threads than elements, SP = blockDim / nE (a power of
// two) threads share an element's chunks (thread s of it sums k = s, s + SP, ...) and the SP partials are added in
// fixed order through `part` (>= blockDim floats).  Fixed summation order throughout.
__device__ __forceinline__ void stage_chunk_sums(const float* __restrict__ slab, int chunks, int C, int b0, int c0,
                                                 int CW, int nE, float scale, float* __restrict__ sm,
                                                 float* __restrict__ part) {
  const int nt = blockDim.x, t = threadIdx.x;
  int sp = 1;
  while (sp * 2 * nE <= nt && sp * 2 <= chunks) sp *= 2;
  if (sp == 1) {
    for (int e0 = t; e0 < nE; e0 += 4 * nt) {
      const float* src[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = min(e0 + u * nt, nE - 1), bb = e / CW, c = c0 + e - bb * CW;
        src[u] = slab + (long)(b0 + bb) * chunks * C + c;
      }
      float a[4][4] = {};
      for (int k = 0; k < chunks; k += 4) {  // chunk k + q into accumulator q (the tail group guarded, not serial)
        float v[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[u][q] = k + q < chunks ? src[u][(long)(k + q) * C] : 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q) a[u][q] += v[u][q];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (e0 + u * nt < nE) sm[e0 + u * nt] = ((a[u][0] + a[u][1]) + (a[u][2] + a[u][3])) * scale;
    }
    return;
  }
  // sp > 1: one (element, share) per thread
  const int e = t % nE, sh = t / nE;
  if (sh < sp) {
    const int bb = e / CW, c = c0 + e - bb * CW;
    const float* src = slab + (long)(b0 + bb) * chunks * C + c;
    float a[4] = {};
    for (int k = sh; k < chunks; k += 4 * sp) {
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = k + q * sp < chunks ? src[(long)(k + q * sp) * C] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += v[q];
    }
    part[sh * nE + e] = (a[0] + a[1]) + (a[2] + a[3]);
  }
  __syncthreads();
  if (t < nE) {
    float v = 0.f;
    for (int j = 0; j < sp; ++j) v += part[j * nE + t];
    sm[t] = v * scale;
  }
}

// SCA forward (NAFNet_arch.py:39-41, 62): mean[b][i] = pool / HW, a[b][o] = bsca[o] + sum_i W[o][i] mean[b][i].
// grid (C / 4, B / NB), 4 waves: each block stages the means of its NB images (blockIdx.x == 0 also stores them for
// the backward), then one wave per output o: the W row is loaded at once (C / 64 <= 16 values per lane), NB dots.
template <int NB>
__global__ __launch_bounds__(256) void sca_gemv(const float* __restrict__ pool, int chunks, float inv_hw,
                                                float* __restrict__ mean_out, const float* __restrict__ wsca,
                                                const float* __restrict__ bsca, float* __restrict__ a_out, int B,
                                                int C) {
  extern __shared__ float sm[];  // [NB][C] then [256] partials
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int o = blockIdx.x * 4 + wv, b0 = blockIdx.y * NB, nb = min(NB, B - b0);
  // the W row: unconditional loads of clamped (in-bounds) indices, entries past C unused by the dot below, so the
  // loads stay in flight with the chunk-sum loads (a guarded / masked copy waited for them first)
  float w[16];
  const long orow = (long)min(o, C - 1) * C;
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = wsca[orow + min(lane + 64 * j, C - 1)];
  stage_chunk_sums(pool, chunks, C, b0, 0, C, nb * C, inv_hw, sm, sm + NB * C);
  __syncthreads();
  if (blockIdx.x == 0)
    for (int e = threadIdx.x; e < nb * C; e += blockDim.x) mean_out[(long)b0 * C + e] = sm[e];
  if (o >= C) return;
  float acc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int i = lane + 64 * j;
    if (i < C)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (b < nb) acc[b] = fmaf(w[j], sm[b * C + i], acc[b]);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const float v = wave_sum(acc[b]);
    if (lane == 0 && b < nb) a_out[(long)(b0 + b) * C + o] = v + bsca[o];
  }
}

// sum over pixels p = p, p + step, ... < p1 of x[o(p)] * y[o(p)] (HASY) or x[o(p)], in ascending p: 8 pixels' loads
// issued before their adds (a load per pixel waited for before the next one was issued, and y's inside its branch
// after x's); the product is rounded before the add as before (no contraction into an fma)
template <bool HASY, typename T>
__device__ __forceinline__ void chan_dot_run(const T* __restrict__ x, const T* __restrict__ y, long base, int C, int p,
                                             int p1, int step, float4& acc) {
  auto prod = [&](float4 v, float4 w) {
    float4 r = v * w;
    asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z), "+v"(r.w));
    return r;
  };
  for (; p + 7 * step < p1; p += 8 * step) {
    float4 v[8], w[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ldq(x + base + (long)(p + u * step) * C);
    if constexpr (HASY) {
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = ldq(y + base + (long)(p + u * step) * C);
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = prod(v[u], w[u]);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
  }
  for (; p < p1; p += step) {
    float4 v = ldq(x + base + (long)p * C);
    if constexpr (HASY) v = prod(v, ldq(y + base + (long)p * C));
    acc += v;
  }
}

// per-image channel reduction: slab[b][chunk][c] = sum_{p in chunk} x[p][c] * (y ? y[p][c] : 1).
// grid (chunks, B, ceil(C / 64) channel groups of up to 64 channels): each block a pixel chunk x channel group.
template <typename T>
__global__ void img_chan_dot(const T* __restrict__ x, const T* __restrict__ y, float* __restrict__ slab, Geo geo) {
  extern __shared__ float red[];
  // channel group blockIdx.z: 64 channels (the last group of a C that is not a multiple of 64: the rest)
  const int C = geo.C, c0 = blockIdx.z * 64, CG = min(64, C - c0), Q = CG / 4;
  const int tid = threadIdx.x, q = tid % Q, pl = tid / Q, PPI = blockDim.x / Q;
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int HW = geo.H * geo.W;
  const int p0 = chunk * geo.chunk_px, p1 = min(HW, p0 + geo.chunk_px);
  float4 acc = f4(0.f);
  if (pl < PPI) {
    const long base = (long)b * HW * C + c0 + q * 4;
    if (y) chan_dot_run<true>(x, y, base, C, p0 + pl, p1, PPI, acc);
    else chan_dot_run<false>(x, y, base, C, p0 + pl, p1, PPI, acc);
  }
  st4(red + tid * 4, acc);
  __syncthreads();
  if (pl == 0) {
    float4 s = f4(0.f);
    for (int k = 0; k < PPI; ++k) s += ld4(red + (k * Q + q) * 4);
    st4(slab + ((long)b * geo.chunks + chunk) * C + c0 + q * 4, s);
  }
}

// SCA backward: ds[b][i] = sum_o W[o][i] da[b][o] (da reduced by reduce_rows8, staged in LDS).  Block = 64 columns
// x SCA_BW waves splitting the o range (4 W loads in flight per lane); fixed-order cross-wave sum.
constexpr int SCA_BW = 16;
__global__ __launch_bounds__(1024) void sca_bwd_ds(const float* __restrict__ da, const float* __restrict__ wsca,
                                                   float* __restrict__ ds_out, int B, int C) {
  extern __shared__ float sh[];  // da [SCA_NB][C] then partials [SCA_BW][SCA_NB][64]
  float* sda = sh;
  float* part = sh + SCA_NB * C;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int b0 = blockIdx.y * SCA_NB, nb = min(SCA_NB, B - b0);
  for (int e0 = threadIdx.x; e0 < SCA_NB * C; e0 += 4 * blockDim.x) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * blockDim.x;
      v[u] = e < nb * C ? da[(long)b0 * C + e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (e0 + u * blockDim.x < SCA_NB * C) sda[e0 + u * blockDim.x] = v[u];
  }
  __syncthreads();
  float acc[SCA_NB];
#pragma unroll
  for (int b = 0; b < SCA_NB; ++b) acc[b] = 0.f;
  const int per = (C + SCA_BW - 1) / SCA_BW, o0 = wv * per, o1 = min(C, o0 + per);
  if (i < C) {
    int o = o0;
    for (; o + 3 < o1; o += 4) {
      float w[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) w[u] = wsca[(long)(o + u) * C + i];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int b = 0; b < SCA_NB; ++b) acc[b] = fmaf(w[u], sda[b * C + o + u], acc[b]);
    }
    for (; o < o1; ++o) {
      const float w = wsca[(long)o * C + i];
#pragma unroll
      for (int b = 0; b < SCA_NB; ++b) acc[b] = fmaf(w, sda[b * C + o], acc[b]);
    }
  }
#pragma unroll
  for (int b = 0; b < SCA_NB; ++b) part[(wv * SCA_NB + b) * 64 + lane] = acc[b];
  __syncthreads();
  for (int e = threadIdx.x; e < nb * 64; e += blockDim.x) {
    const int b = e >> 6, l = e & 63, ii = blockIdx.x * 64 + l;
    if (ii < C) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < SCA_BW; ++w) v += part[(w * SCA_NB + b) * 64 + l];
      ds_out[(long)(b0 + b) * C + ii] = v;
    }
  }
}

// One launch for the SCA backward (NAFNet_arch.py:39-41, 67), 16 waves per block.  Blocks [0, nds): ds[b][i] =
// sum_o W[o][i] da[b][o] for 64 columns i x NB images, the waves splitting the o range (16 W loads in flight per
// lane) and summed in fixed order, da reduced from the img_chan_dot slab in the block itself.  Blocks [nds, nds +
// C/8): the weight gradients of 8 rows o: dW[o][i] = sum_b da[b][o] mean[b][i], db[o] = sum_b da[b][o] (written to
// their final place: no slab, no separate K = B GEMM).  Fixed summation orders throughout.
constexpr int SCA_OB = 8;
template <int NB>
__global__ __launch_bounds__(1024) void sca_bwd_fused(const float* __restrict__ slab, int chunks,
                                                      const float* __restrict__ wsca, const float* __restrict__ mean,
                                                      float* __restrict__ ds_out, float* __restrict__ dW,
                                                      float* __restrict__ db, int B, int C, int nds) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int nt = blockDim.x;
  if ((int)blockIdx.x >= nds) {
    const int o0 = (blockIdx.x - nds) * SCA_OB, no = min(SCA_OB, C - o0);
    float* sda = sh;  // [B][no]
    // thread = column i x a row group (rows rg, rg + G, ...): the mean column is loaded once per 16 images for all of
    // its rows (the first 16 before the da staging, so both latencies overlap); the sum over b runs in ascending order
    const int G = nt / C, i = threadIdx.x % C, rg = threadIdx.x / C;
    const bool act = rg < G && rg < no;
    float m[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) m[u] = act && u < B ? mean[(long)u * C + i] : 0.f;
    stage_chunk_sums(slab, chunks, C, 0, o0, no, B * no, 1.f, sda, sh + B * SCA_OB);
    __syncthreads();
    if (act) {
      float acc[SCA_OB];
#pragma unroll
      for (int k = 0; k < SCA_OB; ++k) acc[k] = 0.f;
      for (int b = 0; b < B; b += 16) {
        if (b > 0)
#pragma unroll
          for (int u = 0; u < 16; ++u) m[u] = b + u < B ? mean[(long)(b + u) * C + i] : 0.f;
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (b + u < B)
#pragma unroll
            for (int k = 0; k < SCA_OB; ++k) {
              const int r = rg + k * G;
              if (r < no) acc[k] = fmaf(sda[(b + u) * no + r], m[u], acc[k]);
            }
      }
#pragma unroll
      for (int k = 0; k < SCA_OB; ++k) {
        const int r = rg + k * G;
        if (r < no) dW[(long)(o0 + r) * C + i] = acc[k];
      }
    }
    if ((int)threadIdx.x < no) {
      float t = 0.f;
      for (int b = 0; b < B; ++b) t += sda[b * no + threadIdx.x];
      db[o0 + threadIdx.x] = t;
    }
    return;
  }
  float* sda = sh;            // [NB][C]
  float* part = sh + NB * C;  // staging partials, then [SCA_BW][NB][64]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ncb = (C + 63) / 64, cb = blockIdx.x % ncb, bt = blockIdx.x / ncb;
  const int i = cb * 64 + lane;
  const int b0 = bt * NB, nb = min(NB, B - b0);
  const int per = (C + SCA_BW - 1) / SCA_BW, o0 = wv * per, o1 = min(C, o0 + per);
  // the first 16 W values of this wave's o range are loaded before the da staging (overlapping latencies)
  float w[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) w[u] = i < C && o0 + u < o1 ? wsca[(long)(o0 + u) * C + i] : 0.f;
  stage_chunk_sums(slab, chunks, C, b0, 0, C, nb * C, 1.f, sda, part);
  __syncthreads();
  float acc[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) acc[b] = 0.f;
  const bool vec = (per & 3) == 0 && (C & 3) == 0;  // o0, o1 multiples of 4: 16-byte LDS reads of 4 da values
  if (i < C) {
    for (int o = o0; o < o1; o += 16) {
      if (o > o0)
#pragma unroll
        for (int u = 0; u < 16; ++u) w[u] = o + u < o1 ? wsca[(long)(o + u) * C + i] : 0.f;
      if (vec) {
#pragma unroll
        for (int u = 0; u < 16; u += 4)
          if (o + u < o1)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              if (b < nb) {
                const float4 d = *reinterpret_cast<const float4*>(sda + b * C + o + u);
                acc[b] = fmaf(w[u], d.x, acc[b]);
                acc[b] = fmaf(w[u + 1], d.y, acc[b]);
                acc[b] = fmaf(w[u + 2], d.z, acc[b]);
                acc[b] = fmaf(w[u + 3], d.w, acc[b]);
              }
      } else {
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (o + u < o1)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              if (b < nb) acc[b] = fmaf(w[u], sda[b * C + o + u], acc[b]);
      }
    }
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) part[(wv * NB + b) * 64 + lane] = acc[b];
  __syncthreads();
  for (int e = threadIdx.x; e < nb * 64; e += nt) {
    const int b = e >> 6, l = e & 63, ii = cb * 64 + l;
    if (ii < C) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < SCA_BW; ++w) v += part[(w * NB + b) * 64 + l];
      ds_out[(long)(b0 + b) * C + ii] = v;
    }
  }
}

// dg = dh * a[b] + ds[b] / HW ; SimpleGate backward: dt2[:C] = dg * t2[C:], dt2[C:] = dg * t2[:C]
template <typename T>
__global__ void sca_sg_bwd(const T* __restrict__ dh, const float* __restrict__ a, const float* __restrict__ ds,
                           const T* __restrict__ t2, T* __restrict__ dt2, long M, int C, int HW, float inv_hw) {
  const int Q = C / 4;
  const long total = M * Q;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long m = e / Q;
    const int q = e % Q;
    const int b = m / HW;
    const float4 dg = fma4(ldq(dh + m * C + q * 4), ld4(a + (long)b * C + q * 4), ld4(ds + (long)b * C + q * 4) * f4(inv_hw));
    const float4 ta = ldq(t2 + m * 2 * C + q * 4), tb = ldq(t2 + m * 2 * C + C + q * 4);
    stq(dt2 + m * 2 * C + q * 4, dg * tb);
    stq(dt2 + m * 2 * C + C + q * 4, dg * ta);
  }
}

// depthwise 3x3 backward on C2 channels: dt1 = sum_t w[t] dt2(p - off_t) ; partial dW[c][t] = sum dt2(p) t1(p+off_t),
// partial db[c] = sum dt2(p).  slab: [B*chunks][C2][10]
template <typename T>
__global__ void dw_bwd(const T* __restrict__ dt2, const T* __restrict__ t1, const float* __restrict__ wdw,
                       T* __restrict__ dt1, float* __restrict__ slab_w, float* __restrict__ slab_b, Geo geo) {
  extern __shared__ float red[];  // [blockDim][4]
  const int C2 = 2 * geo.C, Q = C2 / 4;
  const int tid = threadIdx.x, q = tid % Q, pl = tid / Q, PPI = blockDim.x / Q;
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int HW = geo.H * geo.W;
  float wk[4][9];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int t = 0; t < 9; ++t) wk[j][t] = wdw[(q * 4 + j) * 9 + t];
  float4 aw[9], ab = f4(0.f);
#pragma unroll
  for (int t = 0; t < 9; ++t) aw[t] = f4(0.f);
  const int p0 = chunk * geo.chunk_px, p1 = min(HW, p0 + geo.chunk_px);
  const T* gb = dt2 + (long)b * HW * C2 + q * 4;
  const T* xb = t1 + (long)b * HW * C2 + q * 4;
  if (pl < PPI) {
    for (int p = p0 + pl; p < p1; p += PPI) {
      const int h = p / geo.W, w = p - h * geo.W;
      const float4 gc = ldq(gb + (long)p * C2);
      ab += gc;
      float4 acc = f4(0.f);
#pragma unroll
      for (int dh = -1; dh <= 1; ++dh) {
#pragma unroll
        for (int dw = -1; dw <= 1; ++dw) {
          const int t = (dh + 1) * 3 + (dw + 1);
          // forward: t2(q) += w[t] t1(q + off)  ->  dt1(p) += w[t] dt2(p - off) ; dW[t] += dt2(p) t1(p + off)
          const int hs = h - dh, ws = w - dw;
          if (hs >= 0 && hs < geo.H && ws >= 0 && ws < geo.W) {
            const float4 gv = ldq(gb + ((long)hs * geo.W + ws) * C2);
            acc.x = fmaf(wk[0][t], gv.x, acc.x); acc.y = fmaf(wk[1][t], gv.y, acc.y);
            acc.z = fmaf(wk[2][t], gv.z, acc.z); acc.w = fmaf(wk[3][t], gv.w, acc.w);
          }
          const int hp = h + dh, wp = w + dw;
          if (hp >= 0 && hp < geo.H && wp >= 0 && wp < geo.W) {
            aw[t] = fma4(gc, ldq(xb + ((long)hp * geo.W + wp) * C2), aw[t]);
          }
        }
      }
      stq(dt1 + ((long)b * HW + p) * C2 + q * 4, acc);
    }
  }
  // block reduction over pixel lanes sharing quad q, one tap at a time through a [blockDim][4] buffer
  const long row = (long)b * geo.chunks + chunk;
  float* dw_dst = slab_w + row * C2 * 9;
  float* db_dst = slab_b + row * C2;
#pragma unroll
  for (int t = 0; t < 10; ++t) {
    st4(red + tid * 4, t < 9 ? aw[t] : ab);
    __syncthreads();
    if (pl == 0) {
      float4 sum = f4(0.f);
      for (int k = 0; k < PPI; ++k) sum += ld4(red + (k * Q + q) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (t < 9) dw_dst[(long)(q * 4 + j) * 9 + t] = get(sum, j);
        else db_dst[q * 4 + j] = get(sum, j);
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- LDS-tiled depthwise 3x3 backward
// One block = a TH x TW pixel tile of one image x one 64-byte channel slice (HS gate channels c and their SimpleGate
// partners C + c, so the fused prologue below can form both halves of dt2 from one gate gradient).  The tile plus a
// one-pixel halo of dt2 and t1 is staged once in LDS with 16-byte loads (zeros outside the image = the conv's zero
// padding); each thread then owns one channel quad x one column and walks the TH rows with a 3x3 rolling register
// window, so LDS is read 6 times per output pixel instead of 18 and HBM once per tile (halo re-read 1.2x).
//   dt1(p) = sum_t w[t] dt2(p - off_t) ;  dW[c][t] += dt2(p) t1(p + off_t) ;  db[c] += dt2(p)
// FUSED: dt2 is not materialised; the loader computes dg = dh * a[b] + ds[b] / HW and dt2 = (dg * t2[C:], dg * t2[:C])
// (SCA + SimpleGate backward, NAFNet_arch.py:64-67) straight into LDS.
// Per-tile dW/db partials go to slab row b * tiles + tile (disjoint channel columns per slice), reduced in fixed order.
struct DwTileP {
  const void* dt2;  // [M][2C]           (unfused)
  const void* dh;   // [M][C]            (fused)
  const float* a;   // [B][C]            (fused)
  const float* ds;  // [B][C]            (fused)
  const void* t2;   // [M][2C]           (fused)
  const void* t1;   // [M][2C]
  const float* wdw; // [2C][9]
  const float* bdw; // [2C]               (unused by the backward)
  void* dt1;        // [M][2C]
  float* slab_w;    // [rows][2C][9]
  float* slab_b;    // [rows][2C]
  int B, H, W, C, tiles_x, tiles, slices;
  float inv_hw;
  // SCA: the SCA backward folded in (nbp_sca_dw_bwd): ds of the workgroup's gate channels from the channel-dot slab,
  // and rows of the SCA weight / bias gradients
  const float* da_slab;  // [B][chunks][C]
  const float* wsca;     // [C][C]
  const float* mean;     // [B][C]
  float* dwsca;          // [C][C] out
  float* dbsca;          // [C] out
  int chunks;
};


constexpr int DWT_TH = 16;
inline int dw_bwd_tw(int W) { return W >= 32 ? 32 : 16; }

template <typename T>
__device__ __forceinline__ void ld16f(const T* p, float* f) {
  if constexpr (sizeof(T) == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  } else {
    const vec_t<T, 8> v = *reinterpret_cast<const vec_t<T, 8>*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  }
}
template <typename T>
__device__ __forceinline__ void st16f(T* p, const float* f) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  } else {
    vec_t<T, 8> v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (T)f[j];
    *reinterpret_cast<vec_t<T, 8>*>(p) = v;
  }
}

template <typename T>
__device__ __forceinline__ void unpack16(uint4 r, float* f) {
  if constexpr (sizeof(T) == 4) {
    f[0] = __uint_as_float(r.x); f[1] = __uint_as_float(r.y); f[2] = __uint_as_float(r.z); f[3] = __uint_as_float(r.w);
  } else {
    const vec_t<T, 8> v = __builtin_bit_cast(vec_t<T, 8>, r);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
  }
}

// (A variant that recomputed t2 from t1 in LDS instead of reading it, so that the forward need not store it, measured
// neutral to slower and was removed in round 4.)
template <typename T, bool FUSED, int DWT_TW, bool SCA = false>
__global__ __launch_bounds__(256) void dw_bwd_tiled(DwTileP p) {
  static_assert(!SCA || FUSED, "the SCA fold feeds the fused loader");
  constexpr int E = 16 / sizeof(T);      // elements per 16-byte chunk
  constexpr int CSL = 64 / sizeof(T);    // conv channels per slice
  constexpr int HS = CSL / 2;            // gate channels per slice
  constexpr int NQ = CSL / 4;            // channel quads per slice
  constexpr int NT = NQ * DWT_TW;        // threads
  constexpr int TH = DWT_TH;
  constexpr int LW = DWT_TW + 2, LH = TH + 2;
  __shared__ __attribute__((aligned(16))) T sg[LH * LW * CSL];
  __shared__ __attribute__((aligned(16))) T sx[LH * LW * CSL];
  // t1 at (row, col) of the one-pixel-halo frame
  auto SX = [&](int row, int col) { return sx + (row * LW + col) * CSL; };
  const int tid = threadIdx.x;
  const int u = xcd_remap(blockIdx.x, gridDim.x);  // the slices of one tile share an XCD (and its L2)
  const int slice = u % p.slices, tile = (u / p.slices) % p.tiles, b = u / (p.slices * p.tiles);
  const int y0 = (tile / p.tiles_x) * TH, x0 = (tile % p.tiles_x) * DWT_TW;
  const int C = p.C, C2 = 2 * C, H = p.H, W = p.W;
  const long img = (long)b * H * W;
  const int cbase = slice * HS;
  const int q = tid % NQ, x = tid / NQ;
  const int lc = 4 * q;
  const int gc = lc < HS ? cbase + lc : C + cbase + (lc - HS);
  // the 4 channels' taps as packed pairs {c, c+1}, {c+2, c+3}: every FMA below is a v_pk_fma_f32 on register pairs
  // that already sit together (no per-FMA operand moves)
  f2v wk[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) wk[t][hh] = f2v{p.wdw[(gc + 2 * hh) * 9 + t], p.wdw[(gc + 2 * hh + 1) * 9 + t]};
  // ---- stage t1 (and dt2 when unfused): 4 chunks per pixel = 2 halves x 2 chunks.  Every load of the stage is
  // issued before the first LDS store (register batches): one memory latency per tile instead of one per pass.
  constexpr int TOT2 = LH * LW * 2, N2 = FUSED ? (TOT2 + NT - 1) / NT : 1;
  uint4 rd[N2], ra[N2], rb[N2];
  // addressing: 64-bit element index of the staging frame's origin pixel once per tile, then 32-bit in-frame offsets
  // from 24-bit multiplies (full-rate v_mul_u32_u24; the launcher bounds W * 2C < 2^24) -- no per-load 64-bit or
  // 32 x 32 multiplies
  const unsigned rs1 = (unsigned)W * C2, rsh = (unsigned)W * C;  // row strides (elements) of t1 / t2 / dt1 and dh
  {
    const T* t1 = reinterpret_cast<const T*>(p.t1);
    const T* dt2 = reinterpret_cast<const T*>(p.dt2);
    constexpr int TOT1 = LH * LW * 4, N1 = (TOT1 + NT - 1) / NT;
    const long e1 = (img + (long)(y0 - 1) * W + (x0 - 1)) * C2 + cbase;
    uint4 vx[N1], vg[FUSED ? 1 : N1];
#pragma unroll
    for (int it = 0; it < N1; ++it) {
      const int i = tid + it * NT;
      vx[it] = make_uint4(0, 0, 0, 0);
      if (!FUSED) vg[it] = make_uint4(0, 0, 0, 0);
      const int pix = i >> 2, hh = (i >> 1) & 1, k = i & 1;
      const int py = pix / LW, px = pix % LW;
      const int gy = y0 - 1 + py, gx = x0 - 1 + px;
      if (i < TOT1 && gy >= 0 && gy < H && gx >= 0 && gx < W) {
        const long go = e1 + (long)(__umul24(py, rs1) + __umul24(px, C2) + hh * C + k * E);
        vx[it] = *reinterpret_cast<const uint4*>(t1 + go);
        if (!FUSED) vg[it] = *reinterpret_cast<const uint4*>(dt2 + go);
      }
    }
    if (FUSED) {
      const T* dh = reinterpret_cast<const T*>(p.dh);
      const T* t2 = reinterpret_cast<const T*>(p.t2);
      const long o2 = img + (long)(y0 - 1) * W + (x0 - 1);
      const long eh = o2 * C + cbase, e2 = o2 * C2 + cbase;
#pragma unroll
      for (int it = 0; it < N2; ++it) {
        const int i = tid + it * NT;
        const int pix = i >> 1, k = i & 1;
        const int py = pix / LW, px = pix % LW;
        const int gy = y0 - 1 + py, gx = x0 - 1 + px;
        rd[it] = ra[it] = rb[it] = make_uint4(0, 0, 0, 0);
        if (i < TOT2 && gy >= 0 && gy < H && gx >= 0 && gx < W) {
          rd[it] = *reinterpret_cast<const uint4*>(dh + eh + (long)(__umul24(py, rsh) + __umul24(px, C) + k * E));
          const long o = e2 + (long)(__umul24(py, rs1) + __umul24(px, C2) + k * E);
          ra[it] = *reinterpret_cast<const uint4*>(t2 + o);
          rb[it] = *reinterpret_cast<const uint4*>(t2 + o + C);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < N1; ++it) {
      const int i = tid + it * NT;
      if (i < TOT1) {
        const int pix = i >> 2, hh = (i >> 1) & 1, k = i & 1;
        const int lo = pix * CSL + hh * HS + k * E;
        *reinterpret_cast<uint4*>(sx + lo) = vx[it];
        if (!FUSED) *reinterpret_cast<uint4*>(sg + lo) = vg[it];
      }
    }
  }
  // SCA scratch in the dt2 tile (written only below, after the ds values are in registers; and free again after the
  // final reduction): no LDS of its own, the resident workgroups per CU unchanged
  float* sca_s = reinterpret_cast<float*>(sg);  // part [1024] | sdb [1024] | red [4 NT] | sds [HS]
  static_assert(!SCA || (2048 + 4 * NT + HS) * 4 <= LH * LW * CSL * (int)sizeof(T), "SCA scratch");
  static_assert(!SCA || (NT <= SCA_DW_BMAX && 2 * SCA_DW_BMAX * 4 <= LH * LW * CSL * (int)sizeof(T)), "SCA scratch");
  [[maybe_unused]] const ScaBwdP sq{p.da_slab, p.wsca, p.mean, p.dwsca, p.dbsca, p.chunks, p.B, p.C};
  if constexpr (SCA) sca_ds_slice<NT, HS>(sq, b, cbase, sca_s, sca_s + 1024, sca_s + 2048, sca_s + 2048 + 4 * NT);
  if (FUSED) {
    // NT is even, so this thread's chunk k = tid & 1 (and its E channels) is the same in every pass: a and ds / HW once
    static_assert(NT % 2 == 0, "chunk parity per thread");
    float ak[E], sk[E];
    {
      const int c = cbase + (tid & 1) * E;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        ak[j] = p.a[(long)b * C + c + j];
        if constexpr (SCA) sk[j] = sca_s[2048 + 4 * NT + (tid & 1) * E + j] * p.inv_hw;
        else sk[j] = p.ds[(long)b * C + c + j] * p.inv_hw;
      }
    }
    if constexpr (SCA) __syncthreads();  // every thread holds its ds before the tile overwrites the scratch
#pragma unroll
    for (int it = 0; it < N2; ++it) {
      const int i = tid + it * NT;
      if (i >= TOT2) continue;
      const int pix = i >> 1, k = i & 1;
      const int gy = y0 - 1 + pix / LW, gx = x0 - 1 + pix % LW;
      const bool inside = gy >= 0 && gy < H && gx >= 0 && gx < W;
      float d[E], ta[E], tb[E], lo[E], hi[E];
      unpack16<T>(rd[it], d);
      unpack16<T>(ra[it], ta);
      unpack16<T>(rb[it], tb);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        const float dg = inside ? fmaf(d[j], ak[j], sk[j]) : 0.f;
        lo[j] = dg * tb[j];
        hi[j] = dg * ta[j];
        // the fp32 products are what is rounded to the storage type (the SimpleGate convention of every kernel):
        // left alone the compiler folds some of the mul + convert pairs into one fp16-output v_fma_mix
        asm volatile("" : "+v"(lo[j]), "+v"(hi[j]));
      }
      st16f(sg + pix * CSL + k * E, lo);
      st16f(sg + pix * CSL + HS + k * E, hi);
    }
  }
  lds_barrier();
  // ---- compute: thread = (quad q, column x)
  f2v aw[9][2], ab[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
#pragma unroll
  for (int t = 0; t < 9; ++t) aw[t][0] = aw[t][1] = f2v{0.f, 0.f};
  f2v gw[3][3][2], xw[3][3][2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    ldq2(sg + (0 * LW + x + j) * CSL + lc, gw[1][j][0], gw[1][j][1]);
    ldq2(sg + (1 * LW + x + j) * CSL + lc, gw[2][j][0], gw[2][j][1]);
    ldq2(SX(0, x + j) + lc, xw[1][j][0], xw[1][j][1]);
    ldq2(SX(1, x + j) + lc, xw[2][j][0], xw[2][j][1]);
  }
  // this thread's dt1 column: one 64-bit base; row r at + r * rs1 (a scalar product: r is unrolled, rs1 uniform)
  T* dtp = reinterpret_cast<T*>(p.dt1) + (img + (long)y0 * W + x0 + x) * C2 + gc;
  const bool col_ok = x0 + x < W;
#pragma unroll
  for (int r = 0; r < TH; ++r) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        gw[0][j][hh] = gw[1][j][hh]; gw[1][j][hh] = gw[2][j][hh];
        xw[0][j][hh] = xw[1][j][hh]; xw[1][j][hh] = xw[2][j][hh];
      }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      ldq2(sg + ((r + 2) * LW + x + j) * CSL + lc, gw[2][j][0], gw[2][j][1]);
      ldq2(SX(r + 2, x + j) + lc, xw[2][j][0], xw[2][j][1]);
    }
    f2v acc[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
#pragma unroll
    for (int dh = -1; dh <= 1; ++dh)
#pragma unroll
      for (int dw = -1; dw <= 1; ++dw) {
        const int t = (dh + 1) * 3 + (dw + 1);
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          acc[hh] = __builtin_elementwise_fma(wk[t][hh], gw[1 - dh][1 - dw][hh], acc[hh]);
          aw[t][hh] = __builtin_elementwise_fma(gw[1][1][hh], xw[1 + dh][1 + dw][hh], aw[t][hh]);
        }
      }
    ab[0] += gw[1][1][0];
    ab[1] += gw[1][1][1];
    // the row's dt1 and weight-gradient FMAs are materialised here, in one block: left alone the compiler sinks dt1's
    // two 9-FMA chains into the store's branch (dependent v_pk_fma_f32 back to back, an s_nop between each pair) and
    // every row's dW FMAs past the loop (all rows' windows held raw in registers)
    asm volatile("" : "+v"(acc[0]), "+v"(acc[1]));
    asm volatile("" : "+v"(aw[0][0]), "+v"(aw[0][1]), "+v"(aw[1][0]), "+v"(aw[1][1]), "+v"(aw[2][0]), "+v"(aw[2][1]),
                 "+v"(aw[3][0]), "+v"(aw[3][1]), "+v"(aw[4][0]), "+v"(aw[4][1]));
    asm volatile("" : "+v"(aw[5][0]), "+v"(aw[5][1]), "+v"(aw[6][0]), "+v"(aw[6][1]), "+v"(aw[7][0]), "+v"(aw[7][1]),
                 "+v"(aw[8][0]), "+v"(aw[8][1]), "+v"(ab[0]), "+v"(ab[1]));
    if (col_ok && y0 + r < H) stq(dtp + (unsigned)r * rs1, make_float4(acc[0].x, acc[0].y, acc[1].x, acc[1].y));
  }
  // ---- reduce the 40 partials over the tile's columns: lanes of one quad differ in bits >= log2(NQ)
  float v[40];
#pragma unroll
  for (int t = 0; t < 10; ++t) {
    const f2v a0 = t < 9 ? aw[t][0] : ab[0], a1 = t < 9 ? aw[t][1] : ab[1];
    v[4 * t] = a0.x; v[4 * t + 1] = a0.y; v[4 * t + 2] = a1.x; v[4 * t + 3] = a1.y;
  }
  const int lane = tid & 63, wave = tid >> 6;
  constexpr int NW = NT / 64;
  float* red = reinterpret_cast<float*>(sg);
  if constexpr (NQ == 8) {
    // reduce-scatter over the 8 columns of a wave (lane bits 3..5): each step keeps half of the values and adds the
    // partner's copy of that half (40 -> 20 -> 10 -> 5 values per lane; 35 shuffles instead of 120).  Every sum is
    // own + partner over the same pairs as the butterfly, so the totals are bitwise those of the butterfly.
    float v2[20], v3[10], v4[5];
    const bool b3 = lane & 8, b4 = lane & 16, b5 = lane & 32;
#pragma unroll
    for (int j = 0; j < 20; ++j) {
      const float snd = b3 ? v[j] : v[j + 20], keep = b3 ? v[j + 20] : v[j];
      v2[j] = keep + __shfl_xor(snd, 8, 64);
    }
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const float snd = b4 ? v2[j] : v2[j + 10], keep = b4 ? v2[j + 10] : v2[j];
      v3[j] = keep + __shfl_xor(snd, 16, 64);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const float snd = b5 ? v3[j] : v3[j + 5], keep = b5 ? v3[j + 5] : v3[j];
      v4[j] = keep + __shfl_xor(snd, 32, 64);
    }
    lds_barrier();  // tiles are dead: reuse sg as the cross-wave buffer
    const int e0 = (b3 ? 20 : 0) + (b4 ? 10 : 0) + (b5 ? 5 : 0);
#pragma unroll
    for (int j = 0; j < 5; ++j) red[(wave * NQ + (lane & 7)) * 40 + e0 + j] = v4[j];
  } else {
#pragma unroll
    for (int i = 0; i < 40; ++i)
#pragma unroll
      for (int o = NQ; o < 64; o <<= 1) v[i] += __shfl_xor(v[i], o, 64);
    lds_barrier();  // tiles are dead: reuse sg as the cross-wave buffer
    if (lane < NQ) {
#pragma unroll
      for (int i = 0; i < 40; ++i) red[(wave * NQ + lane) * 40 + i] = v[i];
    }
  }
  lds_barrier();
  const long row = (long)b * p.tiles + tile;
  for (int i = tid; i < NQ * 40; i += NT) {
    const int qq = i / 40, e = i % 40, t = e >> 2, j = e & 3;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[(w * NQ + qq) * 40 + e];
    const int l = 4 * qq + j;
    const int ch = l < HS ? cbase + l : C + cbase + (l - HS);
    if (t < 9) p.slab_w[(row * C2 + ch) * 9 + t] = s;
    else p.slab_b[row * C2 + ch] = s;
  }
  if constexpr (SCA) sca_dw_rows<NT>(sq, sca_s, sca_s + SCA_DW_BMAX);  // (its first barrier: the reduction is done)
}

// ---------------------------------------------------------------- LDS-tiled depthwise 3x3 + SimpleGate + pool partials
// Same tiling as the backward: a TH x TW pixel tile x one 64-byte channel slice (HS gate channels c and partners C + c)
// staged once in LDS with its halo.  Thread = (gate quad, column): it convolves the 4 channels c.. and the 4 partners
// C + c.. with rolling 3x3 register windows, writes t2 (both halves), g = t2[:C] * t2[C:] and accumulates the pool
// partial of g, reduced over the tile into pool_slab[b][tile][C] (fixed order).
struct DwFwdP {
  const void* t1;
  const float* wdw;
  const float* bdw;
  void* t2;
  void* g;
  float* pool_slab;
  int B, H, W, C, tiles_x, tiles, slices;
};
// tile width: 64 / 32 / 16 columns by image width; fp32 (2 gate quads per slice) never below 32 (whole waves)
inline int dw_fwd_tw(int W, int dtype) { return W >= 64 ? 64 : ((W >= 32 || dtype == 0) ? 32 : 16); }
// tile height: 16 rows, 8 at the small deep-level images (W <= 32: 2x the blocks, half of each thread's serial
// row chain; the extra halo rows are L2 hits)
inline int dw_fwd_th(int W) { return W <= 32 ? 8 : DWT_TH; }
int dw_fwd_tiles(int H, int W, int dtype) { return cdiv(H, dw_fwd_th(W)) * cdiv(W, dw_fwd_tw(W, dtype)); }

template <typename T, int TW, int TH = DWT_TH>
__global__ __launch_bounds__(256) void dw_sg_pool_tiled(DwFwdP p) {
  constexpr int E = 16 / sizeof(T), CSL = 64 / sizeof(T), HS = CSL / 2, NQG = HS / 4, NT = NQG * TW;
  constexpr int LW = TW + 2, LH = TH + 2;
  __shared__ __attribute__((aligned(16))) T sx[LH * LW * CSL];
  const int tid = threadIdx.x;
  const int u = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = u % p.slices, tile = (u / p.slices) % p.tiles, b = u / (p.slices * p.tiles);
  const int y0 = (tile / p.tiles_x) * TH, x0 = (tile % p.tiles_x) * TW;
  const int C = p.C, C2 = 2 * C, H = p.H, W = p.W;
  const long img = (long)b * H * W;
  const int cbase = slice * HS;
  const unsigned rs1 = (unsigned)W * C2, rsg = (unsigned)W * C;  // row strides (elements), < 2^24 (launcher)
  {  // all staging loads issued before the LDS stores (one memory latency per tile); 32-bit in-frame offsets
    const T* t1 = reinterpret_cast<const T*>(p.t1);
    constexpr int TOT = LH * LW * 4, N1 = (TOT + NT - 1) / NT;
    const long e1 = (img + (long)(y0 - 1) * W + (x0 - 1)) * C2 + cbase;
    uint4 v[N1];
#pragma unroll
    for (int it = 0; it < N1; ++it) {
      const int i = tid + it * NT;
      const int pix = i >> 2, hh = (i >> 1) & 1, k = i & 1;
      const int py = pix / LW, px = pix % LW;
      const int gy = y0 - 1 + py, gx = x0 - 1 + px;
      v[it] = make_uint4(0, 0, 0, 0);
      if (i < TOT && gy >= 0 && gy < H && gx >= 0 && gx < W)
        v[it] = *reinterpret_cast<const uint4*>(t1 + e1 + (long)(__umul24(py, rs1) + __umul24(px, C2) + hh * C + k * E));
    }
#pragma unroll
    for (int it = 0; it < N1; ++it) {
      const int i = tid + it * NT;
      const int pix = i >> 2, hh = (i >> 1) & 1, k = i & 1;
      if (i < TOT) *reinterpret_cast<uint4*>(sx + pix * CSL + hh * HS + k * E) = v[it];
    }
  }
  lds_barrier();
  const int qg = tid % NQG, x = tid / NQG;
  const int la = 4 * qg, lb = HS + 4 * qg;       // local channels (LDS)
  const int gca = cbase + 4 * qg, gcb = C + gca;  // global conv channels
  // taps of the 4 gate channels (a) and their 4 partners (b) as packed pairs: the FMAs are v_pk_fma_f32 on pairs
  f2v wa[9][2], wb[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      wa[t][hh] = f2v{p.wdw[(gca + 2 * hh) * 9 + t], p.wdw[(gca + 2 * hh + 1) * 9 + t]};
      wb[t][hh] = f2v{p.wdw[(gcb + 2 * hh) * 9 + t], p.wdw[(gcb + 2 * hh + 1) * 9 + t]};
    }
  const float4 ba = ld4(p.bdw + gca), bb = ld4(p.bdw + gcb);
  f2v xa[3][3][2], xb[3][3][2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    ldq2(sx + (0 * LW + x + j) * CSL + la, xa[1][j][0], xa[1][j][1]);
    ldq2(sx + (1 * LW + x + j) * CSL + la, xa[2][j][0], xa[2][j][1]);
    ldq2(sx + (0 * LW + x + j) * CSL + lb, xb[1][j][0], xb[1][j][1]);
    ldq2(sx + (1 * LW + x + j) * CSL + lb, xb[2][j][0], xb[2][j][1]);
  }
  // this thread's column of t2 / g: one 64-bit base each, then a row stride per row
  const long m0 = img + (long)y0 * W + x0 + x;
  T* t2p = p.t2 ? reinterpret_cast<T*>(p.t2) + m0 * C2 : nullptr;
  T* gp = reinterpret_cast<T*>(p.g) + m0 * C;
  float4 pacc = f4(0.f);
  const bool col_ok = x0 + x < W;
#pragma unroll
  for (int r = 0; r < TH; ++r) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        xa[0][j][hh] = xa[1][j][hh]; xa[1][j][hh] = xa[2][j][hh];
        xb[0][j][hh] = xb[1][j][hh]; xb[1][j][hh] = xb[2][j][hh];
      }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      ldq2(sx + ((r + 2) * LW + x + j) * CSL + la, xa[2][j][0], xa[2][j][1]);
      ldq2(sx + ((r + 2) * LW + x + j) * CSL + lb, xb[2][j][0], xb[2][j][1]);
    }
    f2v a2[2] = {f2v{ba.x, ba.y}, f2v{ba.z, ba.w}}, b2[2] = {f2v{bb.x, bb.y}, f2v{bb.z, bb.w}};
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        a2[hh] = __builtin_elementwise_fma(wa[t][hh], xa[t / 3][t % 3][hh], a2[hh]);
        b2[hh] = __builtin_elementwise_fma(wb[t][hh], xb[t / 3][t % 3][hh], b2[hh]);
      }
    const float4 aa = make_float4(a2[0].x, a2[0].y, a2[1].x, a2[1].y);
    const float4 ab = make_float4(b2[0].x, b2[0].y, b2[1].x, b2[1].y);
    if (col_ok && y0 + r < H) {
      if (t2p) {  // null: t2 not kept (no backward follows)
        T* q2 = t2p + (unsigned)r * rs1;
        stq(q2 + gca, aa);
        stq(q2 + gcb, ab);
      }
      float4 gv = aa * ab;
      // the fp32 product is what is rounded to the storage type (as in the other SimpleGate kernels): kept opaque so
      // the mul + convert is not folded into one mixed-precision FMA (one rounding instead of two: other bits)
      asm volatile("" : "+v"(gv.x), "+v"(gv.y), "+v"(gv.z), "+v"(gv.w));
      stq(gp + (unsigned)r * rsg + gca, gv);
      pacc += gv;
    }
  }
  // reduce pacc over the tile's columns (lanes of one gate quad differ in bits >= log2(NQG)), then across waves
#pragma unroll
  for (int o = NQG; o < 64; o <<= 1) {
    pacc.x += __shfl_xor(pacc.x, o, 64); pacc.y += __shfl_xor(pacc.y, o, 64);
    pacc.z += __shfl_xor(pacc.z, o, 64); pacc.w += __shfl_xor(pacc.w, o, 64);
  }
  lds_barrier();
  float* red = reinterpret_cast<float*>(sx);
  const int lane = tid & 63, wave = tid >> 6;
  constexpr int NW = (NT + 63) / 64;
  if (lane < NQG) st4(red + (wave * NQG + lane) * 4, pacc);
  lds_barrier();
  if (tid < NQG * 4) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += red[w * NQG * 4 + tid];
    p.pool_slab[((long)b * p.tiles + tile) * C + cbase + tid] = sum;
  }
}

// backward tile height: 16 rows (8-row tiles were measured neutral at W <= 32 and at every width: DESIGN §5)
int dw_tiles(int H, int W) {
  return cdiv(H, DWT_TH) * cdiv(W, dw_bwd_tw(W));
}
bool dw_tiled_ok(int C, int dtype) { return C % (dtype != 0 ? 16 : 8) == 0; }

int block_for_quads(int Q) {
  if (Q >= 256) return Q;  // one pixel per step, one thread per quad (Q <= 1024)
  return 256;
}

// per-image pixel-chunk budget for the per-image channel reductions (pool, img_chan_dot): chunks of >= 128 pixels,
// at most 64 per image — their consumers re-reduce the partial slab in every block, so it must stay small.
long img_cap(int B, int H, int W) {
  long c = (long)H * W / 128;
  c = c < 1 ? 1 : (c > 64 ? 64 : c);
  return (long)B * c;
}

Geo make_geo(int B, int H, int W, int C, int Q, int block, long cap_blocks) {
  Geo g{B, H, W, C, 1, H * W};
  const int HW = H * W;
  const int ppi = block / Q;
  long want = cap_blocks / B;
  if (want < 1) want = 1;
  long maxc = (HW + ppi - 1) / ppi;  // at least one step per chunk
  if (want > maxc) want = maxc;
  int px = (int)((HW + want - 1) / want);
  px = ((px + ppi - 1) / ppi) * ppi;
  g.chunk_px = px;
  g.chunks = (HW + px - 1) / px;
  return g;
}

int launch_dw_tiled(const void* dt2, const void* dh, const float* a, const float* ds, const void* t2, const void* t1,
                    const float* wdw, const float* bdw, void* dt1, float* dwdw, float* dbdw, float* ws, int B, int H,
                    int W, int C, int dtype, nbp_stream_t s, const DwTileP* sca = nullptr) {
  NBP_REQUIRE((long)W * 2 * C < (1L << 24), "depthwise backward: W * 2C must be < 2^24 (24-bit tile offsets)");
  const int hs = dtype != 0 ? 16 : 8;
  const int tw = dw_bwd_tw(W);
  DwTileP p{dt2, dh, a, ds, t2, t1, wdw, bdw, dt1, nullptr, nullptr, B, H, W, C, cdiv(W, tw), dw_tiles(H, W),
            C / hs, 1.f / (float)(H * W)};
  if (sca) {
    p.da_slab = sca->da_slab; p.wsca = sca->wsca; p.mean = sca->mean; p.dwsca = sca->dwsca; p.dbsca = sca->dbsca;
    p.chunks = sca->chunks;
  }
  const long nrow = (long)B * p.tiles;
  p.slab_w = ws;
  p.slab_b = ws + nrow * 2 * C * 9;
  const long nblk = nrow * p.slices;
  NBP_REQUIRE(nblk < (1L << 31), "dw_bwd: grid too large");
  const bool fused = dh != nullptr;
  lt_begin(S(s));
  NBP_DISPATCH_T(dtype, {
    constexpr int NQ = (64 / sizeof(T)) / 4;
    if (tw == 32) {
      if (sca) dw_bwd_tiled<T, true, 32, true><<<nblk, NQ * 32, 0, S(s)>>>(p);
      else if (fused) dw_bwd_tiled<T, true, 32><<<nblk, NQ * 32, 0, S(s)>>>(p);
      else dw_bwd_tiled<T, false, 32><<<nblk, NQ * 32, 0, S(s)>>>(p);
    } else {
      if (sca) dw_bwd_tiled<T, true, 16, true><<<nblk, NQ * 16, 0, S(s)>>>(p);
      else if (fused) dw_bwd_tiled<T, true, 16><<<nblk, NQ * 16, 0, S(s)>>>(p);
      else dw_bwd_tiled<T, false, 16><<<nblk, NQ * 16, 0, S(s)>>>(p);
    }
  });
  {  // per-launch record (nbp_launch_timing): fused: dh C + t2 2C + t1 2C in, dt1 2C out; else dt2 2C + t1 2C in, dt1 out
    const double M = (double)B * H * W, es = dtype != 0 ? 2 : 4;
    const char* nm = tw == 32 ? (sca ? "dw_bwd_tiled<T,true,32,sca>" : fused ? "dw_bwd_tiled<T,true,32>" : "dw_bwd_tiled<T,false,32>")
                              : (sca ? "dw_bwd_tiled<T,true,16,sca>" : fused ? "dw_bwd_tiled<T,true,16>" : "dw_bwd_tiled<T,false,16>");
    lt_end(S(s), nm, 2.0 * M * 2 * C * 18, (fused ? 7.0 : 6.0) * M * C * es);
  }
  int rc = check_launch("dw_bwd_tiled");
  if (rc) return rc;
  rc = nbp_reduce_slab(p.slab_w, (int)nrow, 2L * C * 9, dwdw, s);
  if (rc) return rc;
  return nbp_reduce_slab(p.slab_b, (int)nrow, 2L * C, dbdw, s);
}

}  // namespace

extern "C" {


// geometry helper for callers sizing the slabs: returns chunks per image for the forward pool / img_chan_dot
int nbp_dw_chunks(int B, int H, int W, int C, int which) {
  // which 0: forward/pool (quads = C/4), 1: dw backward (quads = 2C/4)
  const int Q = which == 0 ? C / 4 : C / 2;
  const int blk = block_for_quads(Q);
  long cap = which == 0 ? img_cap(B, H, W) : (4L << 20) / (2L * C * 10);
  if (cap > 2048) cap = 2048;
  return make_geo(B, H, W, C, Q, blk, cap).chunks;
}

int nbp_dw_fwd_slab_rows(int B, int H, int W, int C, int dtype) {
  if (dw_tiled_ok(C, dtype)) return dw_fwd_tiles(H, W, dtype);
  return nbp_dw_chunks(B, H, W, C, 0);
}

int nbp_dw_sg_pool_fwd(const void* t1, const float* wdw, const float* bdw, void* t2, void* g, float* pool_slab, int B,
                       int H, int W, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(t1 && wdw && bdw && g && pool_slab && B > 0 && H > 0 && W > 0, "nbp_dw_sg_pool_fwd: bad args");
  NBP_REQUIRE(t2 || dw_tiled_ok(C, dtype), "nbp_dw_sg_pool_fwd: t2 may be NULL only on the tiled path (nbp_dw_tiled)");
  NBP_REQUIRE(C % 4 == 0 && C / 4 <= 1024, "nbp_dw_sg_pool_fwd: C");
  if (dw_tiled_ok(C, dtype)) {
    NBP_REQUIRE((long)W * 2 * C < (1L << 24), "nbp_dw_sg_pool_fwd: W * 2C must be < 2^24 (24-bit tile offsets)");
    const int tw = dw_fwd_tw(W, dtype), hs = dtype != 0 ? 16 : 8;
    DwFwdP p{t1, wdw, bdw, t2, g, pool_slab, B, H, W, C, cdiv(W, tw), dw_fwd_tiles(H, W, dtype), C / hs};
    const long nblk = (long)B * p.tiles * p.slices;
    NBP_REQUIRE(nblk < (1L << 31), "nbp_dw_sg_pool_fwd: grid too large");
    NBP_DISPATCH_T(dtype, {
      constexpr int NQG = (32 / sizeof(T)) / 4;
      // whole waves only (the column reduction shuffles across all 64 lanes): fp32 uses TW >= 32
      const int th = dw_fwd_th(W);
      if (tw == 64) dw_sg_pool_tiled<T, 64><<<nblk, NQG * 64, 0, S(s)>>>(p);
      else if ((tw == 32 || NQG * 16 < 64) && th == 8) dw_sg_pool_tiled<T, 32, 8><<<nblk, NQG * 32, 0, S(s)>>>(p);
      else if (tw == 32 || NQG * 16 < 64) dw_sg_pool_tiled<T, 32><<<nblk, NQG * 32, 0, S(s)>>>(p);
      else if (th == 8) dw_sg_pool_tiled<T, 16, 8><<<nblk, NQG * 16, 0, S(s)>>>(p);
      else dw_sg_pool_tiled<T, 16><<<nblk, NQG * 16, 0, S(s)>>>(p);
    });
    return check_launch("dw_sg_pool_tiled");
  }
  const int Q = C / 4, blk = block_for_quads(Q);
  Geo geo = make_geo(B, H, W, C, Q, blk, img_cap(B, H, W));
  dim3 grid(geo.chunks, B);
  NBP_DISPATCH_T(dtype, dw_sg_pool_fwd<T><<<grid, blk, blk * 4 * sizeof(float), S(s)>>>((const T*)t1, wdw, bdw, (T*)t2,
                                                                                       (T*)g, pool_slab, geo));
  return check_launch("dw_sg_pool_fwd");
}

int nbp_sca_fwd(const float* pool_slab, int chunks, const float* wsca, const float* bsca, float* mean, float* a, int B,
                int HW, int C, nbp_stream_t s) {
  NBP_REQUIRE(pool_slab && wsca && bsca && mean && a && B > 0 && C > 0 && chunks > 0, "nbp_sca_fwd: bad args");
  NBP_REQUIRE(C <= 1024, "nbp_sca_fwd: C <= 1024");
  // images per block: the staged chunk sums stay at <= 8 per thread (the loads are latency, not bandwidth)
  int nb = 16;
  while (nb > 1 && (long)nb * C * chunks > 2048) nb /= 2;
  const dim3 grid(cdiv(C, 4), cdiv(B, nb));
  const size_t sm = ((size_t)nb * C + 256) * sizeof(float);
  const float inv = 1.f / (float)HW;
  switch (nb) {
    case 16: sca_gemv<16><<<grid, 256, sm, S(s)>>>(pool_slab, chunks, inv, mean, wsca, bsca, a, B, C); break;
    case 8: sca_gemv<8><<<grid, 256, sm, S(s)>>>(pool_slab, chunks, inv, mean, wsca, bsca, a, B, C); break;
    case 4: sca_gemv<4><<<grid, 256, sm, S(s)>>>(pool_slab, chunks, inv, mean, wsca, bsca, a, B, C); break;
    case 2: sca_gemv<2><<<grid, 256, sm, S(s)>>>(pool_slab, chunks, inv, mean, wsca, bsca, a, B, C); break;
    default: sca_gemv<1><<<grid, 256, sm, S(s)>>>(pool_slab, chunks, inv, mean, wsca, bsca, a, B, C); break;
  }
  return check_launch("sca_fwd");
}

int nbp_img_chan_dot(const void* x, const void* y, float* slab, int B, int H, int W, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && slab && B > 0 && C % 4 == 0 && C / 4 <= 1024, "nbp_img_chan_dot: bad args");
  const int Q = C / 4, blk = block_for_quads(Q);
  Geo geo = make_geo(B, H, W, C, Q, blk, img_cap(B, H, W));  // chunk geometry shared with nbp_dw_chunks(.., 0)
  const int groups = (C + 63) / 64;
  NBP_DISPATCH_T(dtype, img_chan_dot<T><<<dim3(geo.chunks, B, groups), 256, 256 * 4 * sizeof(float), S(s)>>>(
                            (const T*)x, (const T*)y, slab, geo));
  return check_launch("img_chan_dot");
}

int nbp_sca_bwd(const float* da_slab, int chunks, const float* wsca, float* da, float* ds, int B, int C,
                nbp_stream_t s) {
  NBP_REQUIRE(da_slab && wsca && da && ds && B > 0 && C > 0, "nbp_sca_bwd: bad args");
  NBP_REQUIRE(C <= 1024, "nbp_sca_bwd: C <= 1024");
  reduce_rows8<<<cdiv((long)B * C, 32), 256, 0, S(s)>>>(da_slab, B, chunks, C, 1.f, da);
  sca_bwd_ds<<<dim3(cdiv(C, 64), cdiv(B, SCA_NB)), 64 * SCA_BW,
               ((size_t)SCA_NB * C + SCA_BW * SCA_NB * 64) * sizeof(float), S(s)>>>(da, wsca, ds, B, C);
  return check_launch("sca_bwd");
}

int nbp_sca_bwd_fused(const float* da_slab, int chunks, const float* wsca, const float* mean, float* ds, float* dW,
                      float* db, int B, int C, nbp_stream_t s) {
  NBP_REQUIRE(da_slab && wsca && mean && ds && dW && db && B > 0 && C > 0 && chunks > 0, "nbp_sca_bwd_fused: bad args");
  NBP_REQUIRE(C <= 1024 && B <= 4096, "nbp_sca_bwd_fused: C <= 1024, B <= 4096");
  // images per ds block: <= 8 staged chunk loads per thread, at most 4
  int nb = 16;
  while (nb > 1 && (long)nb * C * chunks > 8192) nb /= 2;
  if (nb > 4) nb = 4;  // the per-wave FMA / LDS work grows with nb, the W re-reads (L2) shrink
  const int nds = cdiv(C, 64) * cdiv(B, nb), ndw = cdiv(C, SCA_OB);
  const size_t sm_ds = ((size_t)nb * C + (size_t)SCA_BW * nb * 64 + 1024) * sizeof(float);
  const size_t sm_dw = ((size_t)B * SCA_OB + 1024) * sizeof(float);
  const size_t sm = sm_ds > sm_dw ? sm_ds : sm_dw;
  NBP_REQUIRE(sm <= 160 * 1024, "nbp_sca_bwd_fused: LDS");
  const int g = nds + ndw, ndsx = nds;
  switch (nb) {
    case 16: sca_bwd_fused<16><<<g, 64 * SCA_BW, sm, S(s)>>>(da_slab, chunks, wsca, mean, ds, dW, db, B, C, ndsx); break;
    case 8: sca_bwd_fused<8><<<g, 64 * SCA_BW, sm, S(s)>>>(da_slab, chunks, wsca, mean, ds, dW, db, B, C, ndsx); break;
    case 4: sca_bwd_fused<4><<<g, 64 * SCA_BW, sm, S(s)>>>(da_slab, chunks, wsca, mean, ds, dW, db, B, C, ndsx); break;
    case 2: sca_bwd_fused<2><<<g, 64 * SCA_BW, sm, S(s)>>>(da_slab, chunks, wsca, mean, ds, dW, db, B, C, ndsx); break;
    default: sca_bwd_fused<1><<<g, 64 * SCA_BW, sm, S(s)>>>(da_slab, chunks, wsca, mean, ds, dW, db, B, C, ndsx); break;
  }
  return check_launch("sca_bwd_fused");
}

int nbp_sca_sg_bwd(const void* dh, const float* a, const float* ds, const void* t2, void* dt2, long M, int C, int HW,
                   int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dh && a && ds && t2 && dt2 && M > 0 && C % 4 == 0 && HW > 0, "nbp_sca_sg_bwd: bad args");
  const long tot = M * (C / 4);
  const int gr = cdiv(tot, 256) > 4096 ? 4096 : cdiv(tot, 256);
  NBP_DISPATCH_T(dtype, sca_sg_bwd<T><<<gr, 256, 0, S(s)>>>((const T*)dh, a, ds, (const T*)t2, (T*)dt2, M, C, HW,
                                                            1.f / (float)HW));
  return check_launch("sca_sg_bwd");
}

size_t nbp_dw_bwd_workspace_floats(int B, int H, int W, int C) {
  const size_t a = (size_t)B * nbp_dw_chunks(B, H, W, C, 1), t = (size_t)B * dw_tiles(H, W);
  return (a > t ? a : t) * 2 * C * 10;
}

int nbp_dw_bwd(const void* dt2, const void* t1, const float* wdw, void* dt1, float* dwdw, float* dbdw, float* ws,
               int B, int H, int W, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dt2 && t1 && wdw && dt1 && dwdw && dbdw && ws && B > 0 && C % 2 == 0, "nbp_dw_bwd: bad args");
  if (dw_tiled_ok(C, dtype)) return launch_dw_tiled(dt2, nullptr, nullptr, nullptr, nullptr, t1, wdw, nullptr, dt1, dwdw,
                                                     dbdw, ws, B, H, W, C, dtype, s);
  const int Q = C / 2;  // quads over 2C channels
  NBP_REQUIRE(Q <= 1024, "nbp_dw_bwd: too many channels");
  const int blk = block_for_quads(Q);
  long cap = (4L << 20) / (2L * C * 10);
  if (cap > 2048) cap = 2048;
  Geo geo = make_geo(B, H, W, C, Q, blk, cap);
  const long nrow = (long)B * geo.chunks;
  float* slab_w = ws;
  float* slab_b = ws + nrow * 2 * C * 9;
  NBP_DISPATCH_T(dtype, dw_bwd<T><<<dim3(geo.chunks, B), blk, (size_t)blk * 4 * sizeof(float), S(s)>>>(
                            (const T*)dt2, (const T*)t1, wdw, (T*)dt1, slab_w, slab_b, geo));
  int rc = check_launch("dw_bwd");
  if (rc) return rc;
  rc = nbp_reduce_slab(slab_w, (int)nrow, 2L * C * 9, dwdw, s);
  if (rc) return rc;
  return nbp_reduce_slab(slab_b, (int)nrow, 2L * C, dbdw, s);
}

// SCA + SimpleGate backward fused into the depthwise backward (dt2 never materialised):
// dt2 = (dg * t2[C:], dg * t2[:C]) with dg = dh * a[b] + ds[b] / HW, then dt1 / dW / db as nbp_dw_bwd.
int nbp_sca_sg_dw_bwd(const void* dh, const float* a, const float* ds, const void* t2, const void* t1, const float* wdw,
                      void* dt1, float* dwdw, float* dbdw, float* ws, int B, int H, int W, int C, int dtype,
                      nbp_stream_t s) {
  NBP_REQUIRE(dh && a && ds && t2 && t1 && wdw && dt1 && dwdw && dbdw && ws && B > 0 && H > 0 && W > 0,
              "nbp_sca_sg_dw_bwd: bad args");
  NBP_REQUIRE(dw_tiled_ok(C, dtype), "nbp_sca_sg_dw_bwd: C must be a multiple of %d", dtype != 0 ? 16 : 8);
  return launch_dw_tiled(nullptr, dh, a, ds, t2, t1, wdw, nullptr, dt1, dwdw, dbdw, ws, B, H, W, C, dtype, s);
}

int nbp_dw_tiled(int C, int dtype) { return dw_tiled_ok(C, dtype) ? 1 : 0; }

// The SCA backward folded into the fused depthwise backward: nbp_sca_bwd_fused + nbp_sca_sg_dw_bwd in one launch.
int nbp_sca_dw_bwd(const void* dh, const float* a, const float* da_slab, int chunks, const float* wsca, const float* mean,
                   float* dwsca, float* dbsca, const void* t2, const void* t1, const float* wdw, void* dt1, float* dwdw,
                   float* dbdw, float* ws, int B, int H, int W, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(dh && a && da_slab && wsca && mean && dwsca && dbsca && t2 && t1 && wdw && dt1 && dwdw && dbdw && ws &&
                  B > 0 && H > 0 && W > 0 && chunks > 0,
              "nbp_sca_dw_bwd: bad args");
  NBP_REQUIRE(dw_tiled_ok(C, dtype) && dtype != 0, "nbp_sca_dw_bwd: 16-bit, C a multiple of 16");
  NBP_REQUIRE(C <= 1024 && B <= SCA_DW_BMAX, "nbp_sca_dw_bwd: C <= 1024, B <= %d", SCA_DW_BMAX);
  DwTileP q{};
  q.da_slab = da_slab; q.wsca = wsca; q.mean = mean; q.dwsca = dwsca; q.dbsca = dbsca; q.chunks = chunks;
  return launch_dw_tiled(nullptr, dh, a, nullptr, t2, t1, wdw, nullptr, dt1, dwdw, dbdw, ws, B, H, W, C, dtype, s, &q);
}


}  // extern "C"
