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

#ifdef NBP_GEMM_PROBE
// a trivial kernel that stamps its workgroups' start (slot 0) and XCC_ID (slot 7) into the probe array from row `row0`
__global__ void probe_stamp_kernel(int row0) {
  if (threadIdx.x == 0) {
    const unsigned w = row0 + blockIdx.x;
    if (w < GEMM_PROBE_WGS) {
      g_gemm_probe[w * 8 + 0] = __builtin_amdgcn_s_memrealtime();
      g_gemm_probe[w * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
      g_gemm_probe[w * 8 + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
  }
}
extern "C" int nbp_probe_stamp(int row0, int grid, hipStream_t s) {
  probe_stamp_kernel<<<grid, 256, 0, s>>>(row0);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// the probe library's read-back of the fp16 tiles' timeline (scripts/gemm_timeline.py)
extern "C" int nbp_gemm_probe_read(unsigned long long* host, int words) {
  if (words > GEMM_PROBE_WGS * 8) words = GEMM_PROBE_WGS * 8;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gemm_probe), (size_t)words * 8, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return words;
}
#endif
