// The SCA backward folded into the depthwise backward kernels (nbp_sca_dw_bwd, nbp_sca_c1dw_bwd_tile): each workgroup
// forms ds of its own gate channels from the channel-dot partials, and rows of the SCA weight / bias gradients.
#pragma once
#include "nbp_common.h"

namespace nbp {
namespace {

struct ScaBwdP {
  const float* da_slab;  // [B][chunks][C]: per-chunk partials of sum_p dh (.) g
  const float* wsca;     // [C][C] sca.1.weight
  const float* mean;     // [B][C] the pooled means of the forward
  float* dwsca;          // [C][C] out
  float* dbsca;          // [C] out
  int chunks, B, C;
};

// SCA backward pieces (NAFNet_arch.py:39-41, 67; the arithmetic of sca_bwd_fused, fixed orders of their own):
// da[b][o] = sum over the image's chunks of the slab, ds[b][i] = sum_o W[o][i] da[b][o], dW[o][i] = sum_b da[b][o]
// mean[b][i], db[o] = sum_b da[b][o].  Every piece is laid out for loads in flight (a dependent chain of L2 round trips
// per workgroup cost more than the launch it replaces): the chunk sums split over thread groups with 8 independent
// loads per step, the GEMV over float4 W quads with a thread's loads issued together.

// sum of n values v[k0], v[k0 + step], ... (k < n) of a strided array, 8 loads in flight, fixed order
__device__ __forceinline__ float strided_sum(const float* __restrict__ v, long stride, int k0, int step, int n) {
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = k0;
  for (; k + 7 * step < n; k += 8 * step) {
    float t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = v[(long)(k + q * step) * stride];
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q] += t[q];
  }
  for (int q = 0; k < n; k += step, ++q) a[q] += v[(long)k * stride];
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// ds of the HS gate channels cbase .. of image b into sds.  Scratch: part (max(NT, C) floats), sdb (C), red (NT * 4)
template <int NT, int HS>
__device__ void sca_ds_slice(const ScaBwdP& p, int b, int cbase, float* part, float* sdb, float* red, float* sds) {
  const int tid = threadIdx.x, C = p.C, chunks = p.chunks;
  // da[b][o]: thread (o0 = tid % OW, kg = tid / OW) sums chunks kg, kg + KG, ... of o = o0, o0 + OW, ...
  const int OW = C < NT ? C : NT, KG = NT / OW;
  const float* sl = p.da_slab + (long)b * chunks * C;
  const int o0 = tid % OW, kg = tid / OW;
  if (kg < KG)
    for (int o = o0; o < C; o += OW) part[kg * C + o] = strided_sum(sl + o, C, kg, KG, chunks);
  __syncthreads();
  for (int o = tid; o < C; o += NT) {
    float t = 0.f;
    for (int g = 0; g < KG; ++g) t += part[g * C + o];
    sdb[o] = t;
  }
  __syncthreads();
  // ds: thread (quad qd of the HS channels, o group og) over o = og, og + NG, ...: float4 W loads, 8 at once
  constexpr int NQ4 = HS / 4, NG = NT / NQ4;
  static_assert(HS % 4 == 0 && NT % NQ4 == 0, "SCA GEMV geometry");
  const int qd = tid % NQ4, og = tid / NQ4;
  const float* wq = p.wsca + cbase + 4 * qd;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int o = og; o < C; o += 8 * NG) {
    float4 w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) w[q] = o + q * NG < C ? ld4(wq + (long)(o + q * NG) * C) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float d = o + q * NG < C ? sdb[o + q * NG] : 0.f;
      acc.x = fmaf(w[q].x, d, acc.x);
      acc.y = fmaf(w[q].y, d, acc.y);
      acc.z = fmaf(w[q].z, d, acc.z);
      acc.w = fmaf(w[q].w, d, acc.w);
    }
  }
  reinterpret_cast<float4*>(red)[og * NQ4 + qd] = acc;
  __syncthreads();
  if (tid < HS) {
    float v = 0.f;
    for (int g = 0; g < NG; ++g) v += red[g * HS + tid];
    sds[tid] = v;
  }
  __syncthreads();
}
// the SCA weight / bias gradient rows o = blockIdx.x, + gridDim.x, ...  Scratch: part (max(NT, B) <= SCA_DW_BMAX floats:
// KG * B <= NT when B < NT, else B), sdo (B)
template <int NT>
__device__ void sca_dw_rows(const ScaBwdP& p, float* part, float* sdo) {
  const int tid = threadIdx.x, C = p.C, B = p.B, chunks = p.chunks;
  const int BW = B < NT ? B : NT, KG = NT / BW;  // thread (image bb0 = tid % BW, chunk group kg = tid / BW)
  const int bb0 = tid % BW, kg = tid / BW;
  for (int o = blockIdx.x; o < C; o += gridDim.x) {
    __syncthreads();  // scratch free
    if (kg < KG)
      for (int bb = bb0; bb < B; bb += BW)
        part[kg * B + bb] = strided_sum(p.da_slab + (long)bb * chunks * C + o, C, kg, KG, chunks);
    __syncthreads();
    for (int bb = tid; bb < B; bb += NT) {
      float t = 0.f;
      for (int g = 0; g < KG; ++g) t += part[g * B + bb];
      sdo[bb] = t;
    }
    __syncthreads();
    // 4 columns per thread at once, 16 images each: 64 mean loads in flight (a column at a time left 2 x 4 dependent
    // round trips at the end of every workgroup); the sum over b ascending
    for (int i0 = tid; i0 < C; i0 += 4 * NT) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int b0 = 0; b0 < B; b0 += 16) {
        float m[4][16];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int i = i0 + u * NT;
            m[u][q] = i < C && b0 + q < B ? p.mean[(long)(b0 + q) * C + i] : 0.f;
          }
#pragma unroll
        for (int q = 0; q < 16; ++q)
          if (b0 + q < B)
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] = fmaf(sdo[b0 + q], m[u][q], acc[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i0 + u * NT < C) p.dwsca[(long)o * C + i0 + u * NT] = acc[u];
    }
    if (tid == 0) {
      float t = 0.f;
      for (int bb = 0; bb < B; ++bb) t += sdo[bb];
      p.dbsca[o] = t;
    }
  }
}
constexpr int SCA_DW_BMAX = 256;  // images (the dW rows' da staging)

}  // namespace
}  // namespace nbp
