// Row-ring helpers shared by the row-walking depthwise kernels (c1dw_tile.hip: the level-0/1 tiles with the tape on
// chip; dw_stream.hip: the stored-tape depthwise backward): buffer-descriptor memory operations with out-of-range
// offsets instead of guarded branches, the XOR quad keys of the fp32 LDS rings, packed depthwise taps, the partner-lane
// exchange and compile-time slot indices.
#pragma once
#include <type_traits>

#include "nbp_common.h"

namespace nbp {
namespace {

// Thread map of the depthwise phases (both kernels): lane l of wave w owns the channel quad Q16 = (l & 7) + 8 (l >> 5)
// of the slice (quads 0..7: gate channels, 8..15: their SimpleGate partners, so a gate quad and its partner sit in
// lanes l and l ^ 32 and meet by one shuffle) and PXT adjacent tile columns starting at PXT (4 w + ((l >> 3) & 3)).
// t1 ring rows: LW pixels x 64 fp32 channels (16 quads, 256 B: every pixel starts on bank 0); quad q of pixel px is
// stored at q ^ key(px), a linear XOR key of the pixel's low bits chosen (by exhaustive search over the lane groups of
// ds_read_b128 and ds_write_b128) so that the 16 lanes of a depthwise-phase read (4 column groups PXT apart x 4 quads)
// and the 8 lanes of an MFMA-epilogue write (8 consecutive pixels, one quad) all hit distinct 4-bank quarters.
//
// Memory operations: every global load / store goes through a buffer descriptor of its tensor, with the byte offset
// replaced by OOB (past every descriptor's range) where the pixel lies outside the image: the hardware then returns
// zeros / drops the store.  No memory operation sits behind a data-dependent branch, so the compiler's vmcnt
// accounting stays exact and the rows prefetched into the register rings (static slots: the row loops are unrolled by
// the ring depth, no register copies of in-flight loads) stay in flight across the steps.
template <int PXT>
__device__ __forceinline__ int qkey(int px) {
  if constexpr (PXT == 2) return (px & 1) | ((px & 2) << 2) | ((px & 4) >> 1);  // px bits 0,1,2 -> key bits 0,3,1
  else return (px & 3) | ((px & 4) << 1);                                      // px bits 0,1,2 -> key bits 0,1,3
}

constexpr int OOB = 0x7fffff00;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <typename T>
__device__ __forceinline__ vec_t<T, 8> bload8(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(vec_t<T, 8>, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
template <typename T>
__device__ __forceinline__ vec_t<T, 4> bload4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(vec_t<T, 4>, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
template <typename T>
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, int off, float4 v) {
  vec_t<T, 4> o;
  o[0] = (T)v.x; o[1] = (T)v.y; o[2] = (T)v.z; o[3] = (T)v.w;
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), r, off, 0, 0);
}
template <typename T>
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, int off, vec_t<T, 4> o) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), r, off, 0, 0);
}

// the depthwise taps of one channel quad as packed pairs, and its bias
struct DwQuad {
  f2v w[9][2];
  float4 b;
  __device__ __forceinline__ void load(const float* wdw, const float* bdw, int ch) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 2; ++j) w[t][j] = f2v{wdw[(ch + 2 * j) * 9 + t], wdw[(ch + 2 * j + 1) * 9 + t]};
    b = ld4(bdw + ch);
  }
};

__device__ __forceinline__ float4 f4of(const f2v* v) { return make_float4(v[0].x, v[0].y, v[1].x, v[1].y); }
// the value of lane l ^ 32 (the partner quad's) by one v_permlane32_swap per element: lanes 0..31 read the swapped
// source copy (the upper half's values), lanes 32..63 the swapped destination copy (the lower half's)
__device__ __forceinline__ float swap32(float v, bool upper) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(upper ? r[0] : r[1]);
}
__device__ __forceinline__ float4 swap32(float4 v, bool upper) {
  return make_float4(swap32(v.x, upper), swap32(v.y, upper), swap32(v.z, upper), swap32(v.w, upper));
}

template <int V>
using IC = std::integral_constant<int, V>;

// two fp32 values rounded to the storage type and widened back (v_cvt_pk_{f16,bf16}_f32: round to nearest even, the
// scalar conversion's rounding, two values per instruction)
template <typename T>
__device__ __forceinline__ f2v round2(f2v v) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_convertvector(__builtin_convertvector(v, t2), f2v);
}

}  // namespace
}  // namespace nbp
