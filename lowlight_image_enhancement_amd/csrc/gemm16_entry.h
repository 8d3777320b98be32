// nbp_gemm_bf16's tile dispatch for one 16-bit operand type H, compiled in its own translation unit per type
// (gemm16_bf16.hip, gemm16_fp16.hip).  Returns 1 when the skinny kernel served the call, 0 when a tiled kernel was
// launched, a negative NBP error code otherwise.
#pragma once
#include "nbp_common.h"

namespace nbp {
#define NBP_GEMM16_ENTRY_ARGS                                                                                        \
  const void *A, long lda, int a_mode, const float *a_scale, int rows_per_img, int a_dtype, const void *Bw, long ldb, \
      void *C, long ldc, int c_mode, int c_dtype, int M, int N, int K, int gh, int gw, int cs, const float *bias,     \
      const void *R, const float *rscale, void *pre, hipStream_t st
int gemm16_entry_bf16(NBP_GEMM16_ENTRY_ARGS);
int gemm16_entry_fp16(NBP_GEMM16_ENTRY_ARGS);
}  // namespace nbp
