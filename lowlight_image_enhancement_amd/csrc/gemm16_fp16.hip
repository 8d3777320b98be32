// nbp_gemm_bf16's tile dispatch for the 16-bit operand type fp16 (see gemm16_entry.h)
#include "gemm16_impl.h"
#include "gemm16_entry.h"

namespace nbp {
int gemm16_entry_fp16(NBP_GEMM16_ENTRY_ARGS) {
  using H = _Float16;
  const bool h16 = a_dtype != 0 && c_dtype != 0;
  if (h16 &&
      try_skinny<H>(A, lda, a_mode, a_scale, rows_per_img, Bw, ldb, C, ldc, c_mode, M, N, K, bias, R, rscale, pre, st))
    return 1;
  if (!C) return NBP_ERR_ARG;
  const GemmPB p{A, lda, a_scale, rows_per_img, Bw, ldb, C, ldc, M, N, K, gh, gw, cs, bias, R, rscale, pre};
  if (a_dtype == 0 && c_dtype == 0) return dispatch_modes<float, float, H>(p, a_mode, c_mode, st);
  if (h16) return dispatch_modes<H, H, H>(p, a_mode, c_mode, st);
  if (a_dtype == 0) return dispatch_modes<float, H, H>(p, a_mode, c_mode, st);
  return dispatch_modes<H, float, H>(p, a_mode, c_mode, st);
}
}  // namespace nbp
