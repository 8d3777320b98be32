// Shared device/host helpers for the NewBP-NAFNet MI355X kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/nbp.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// N-element vector of T (T = float, __bf16 or _Float16: the 16-bit storage / MFMA-operand types)
template <typename T, int N>
using vec_t = T __attribute__((ext_vector_type(N)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

namespace nbp {

// ---------------------------------------------------------------- error plumbing (host)
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// per-launch timing records (capi.hip, nbp_launch_timing): events around one kernel launch on stream st
void lt_begin(hipStream_t st);
void lt_end(hipStream_t st, const char* name, double flops, double bytes);
// fp32 implicit-GEMM KH x KW / stride conv over NHWC maps (gemm.hip): mode 0 bias + ReLU, 1 bias, 2 ReLU-mask by R
int conv_f32(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int KH, int KW, int stride, int pad,
             const float* bias, int mode, const float* R, float* y, hipStream_t st);

#define NBP_REQUIRE(cond, ...)            \
  do {                                    \
    if (!(cond)) {                        \
      ::nbp::set_error(__VA_ARGS__);      \
      return NBP_ERR_ARG;                 \
    }                                     \
  } while (0)

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 operator+(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 operator-(float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ float4 operator*(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
__device__ __forceinline__ float4& operator+=(float4& a, float4 b) { a = a + b; return a; }
__device__ __forceinline__ float4 fma4(float4 a, float4 b, float4 c) {
  return make_float4(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z), fmaf(a.w, b.w, c.w));
}
__device__ __forceinline__ float get(float4 v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }
// packed fp32 pair (an adjacent VGPR pair: the operand of v_pk_fma_f32 / v_pk_add_f32)
typedef float f2v __attribute__((ext_vector_type(2)));

// storage-type generic quad (4 consecutive channels) access: fp32 or 16-bit (bf16 / fp16) storage, fp32 math
template <typename T>
__device__ __forceinline__ float4 ldq(const T* p) {
  if constexpr (sizeof(T) == 4) {
    return *reinterpret_cast<const float4*>(p);
  } else {
    const vec_t<T, 4> v = *reinterpret_cast<const vec_t<T, 4>*>(p);
    return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
  }
}
// the same quad as two packed pairs {c, c+1}, {c+2, c+3}
template <typename T>
__device__ __forceinline__ void ldq2(const T* p, f2v& lo, f2v& hi) {
  const float4 v = ldq(p);
  lo = f2v{v.x, v.y};
  hi = f2v{v.z, v.w};
}
template <typename T>
__device__ __forceinline__ void stq(T* p, float4 v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = v;
  } else {
    vec_t<T, 4> o;
    o[0] = (T)v.x; o[1] = (T)v.y; o[2] = (T)v.z; o[3] = (T)v.w;
    *reinterpret_cast<vec_t<T, 4>*>(p) = o;
  }
}

// 32x32x16 MFMA on 16-bit operands (8 per lane), fp32 accumulation: bf16 or fp16 by the operand type
__device__ __forceinline__ floatx16 mfma32x32x16(vec_t<__bf16, 8> a, vec_t<__bf16, 8> b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ floatx16 mfma32x32x16(vec_t<_Float16, 8> a, vec_t<_Float16, 8> b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
// ds_read_b64_tr_b16 for either 16-bit type (the transpose is type-agnostic)
template <typename H>
__device__ __forceinline__ vec_t<H, 4> ds_read_tr16(const H* lds) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lds);
  return __builtin_bit_cast(vec_t<H, 4>, v);
}
template <typename T>
__device__ __forceinline__ float lds1(const T* p) { return (float)*p; }
template <typename T>
__device__ __forceinline__ void sts1(T* p, float v) { *p = (T)v; }

// dtype code of the C-ABI: 0 fp32, 1 bf16, 2 fp16 (the reference's autocast dtype)
#define NBP_DISPATCH_T(dtype, ...)                   \
  do {                                               \
    if ((dtype) == 0) {                              \
      using T = float;                               \
      __VA_ARGS__;                                   \
    } else if ((dtype) == 1) {                       \
      using T = __bf16;                              \
      __VA_ARGS__;                                   \
    } else {                                         \
      using T = _Float16;                            \
      __VA_ARGS__;                                   \
    }                                                \
  } while (0)
// 16-bit storage only: 1 bf16, 2 fp16, as the type alias TN
#define NBP_DISPATCH_16(dtype, TN, ...)              \
  do {                                               \
    if ((dtype) == 2) {                              \
      using TN = _Float16;                           \
      __VA_ARGS__;                                   \
    } else {                                         \
      using TN = __bf16;                             \
      __VA_ARGS__;                                   \
    }                                                \
  } while (0)
#define NBP_DISPATCH_H(dtype, ...) NBP_DISPATCH_16(dtype, H, __VA_ARGS__)
// every storage type (0 fp32, 1 bf16, 2 fp16) as the type alias TN
#define NBP_DISPATCH_ALL(dtype, TN, ...)             \
  do {                                               \
    if ((dtype) == 0) {                              \
      using TN = float;                              \
      __VA_ARGS__;                                   \
    } else {                                         \
      NBP_DISPATCH_16(dtype, TN, __VA_ARGS__);       \
    }                                                \
  } while (0)

// sum over the 64 lanes of a wave
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// sum over aligned groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of one value per thread (blockDim.x multiple of 64, <= 1024); result valid in all threads
__device__ __forceinline__ double block_sum_d(double v, double* red /*>=16*/) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// Workgroups are dealt round-robin to the 8 XCDs (each with its own L2).  Remap the linear block id so that runs of
// consecutive LOGICAL ids land on one XCD: blocks that share input cache lines (e.g. channel slices of one pixel tile)
// then hit the same L2.  Bijective on [0, T): the last T % 8 blocks keep their id.
__device__ __forceinline__ int xcd_remap(int L, int T) {
  const int T8 = T & ~7;
  if (L >= T8) return L;
  return (L & 7) * (T8 >> 3) + (L >> 3);
}

// ---- LDS-DMA (global_load_lds): the LDS destination is wave-uniform base + lane * size; each lane's SOURCE address is
// free, so swizzled LDS images are made by permuting the sources.  Out-of-range lanes read g_zero16 (per-TU zero page).
namespace {
__device__ __attribute__((aligned(16))) unsigned char g_zero16[16];
}
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;
__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((glob_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const void* src, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((glob_void_t*)src, (lds_void_t*)lds_wave_base, 4, 0, 0);
}
// counted wait on this wave's outstanding vector-memory operations (LDS-DMA included)
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// workgroup barrier for LDS hand-offs: waits for this wave's LDS operations only.  __syncthreads' release fence is an
// s_waitcnt vmcnt(0) as well, which exposes the latency of every global store the wave still has in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
inline hipStream_t S(nbp_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace nbp
