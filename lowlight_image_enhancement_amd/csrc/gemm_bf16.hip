// bf16-operand MFMA GEMM (perf mode): C = A(M,K) . W(N,K)^T with fp32 accumulation, v_mfma_f32_32x32x16_bf16.
// The reference trains under AMP (image_restoration_model.py:255, GradScaler :104-106): its convs take half-precision
// operands; here the operands are bf16 (no loss scaling needed: 8-bit exponent), accumulation and epilogue fp32.
// A may be stored fp32 (converted in the tile loader) or bf16; C/R/pre fp32 or bf16.  Same A/C modes as gemm.hip
// (space-to-depth gather for the down conv / up-conv dgrad, per-image column scale for SCA, depth-to-space scatter
// + residual for the up conv).  Weights come from a per-step bf16 copy of the flat parameter buffer; dgrads use
// the transposed copy so every launch is NT.
#include "gemm16_impl.h"
#include "gemm16_entry.h"

extern "C" {

int nbp_gemm_bf16(const void* A, long lda, int a_mode, const float* a_scale, int rows_per_img, int a_dtype,
                  const void* Bw, long ldb, void* C, long ldc, int c_mode, int c_dtype, int M, int N, int K, int gh,
                  int gw, int cs, const float* bias, const void* R, const float* rscale, void* pre, nbp_stream_t s) {
  NBP_REQUIRE(A && Bw && M > 0 && N > 0 && K > 0, "nbp_gemm_bf16: null pointer or empty shape");
  NBP_REQUIRE(a_dtype >= 0 && a_dtype <= 2 && c_dtype >= 0 && c_dtype <= 2 &&
              (a_dtype == 0 || c_dtype == 0 || a_dtype == c_dtype), "nbp_gemm_bf16: dtype");
  // the 16-bit operand type (weights Bw and any 16-bit A / C): fp16 when either side is fp16, else bf16
  const int hd = (a_dtype == 2 || c_dtype == 2) ? 2 : 1;
  const bool h16 = a_dtype != 0 && c_dtype != 0;
  // C may be null only for the skinny SimpleGate forward (the gate input is then recomputed by the backward)
  NBP_REQUIRE(C || (c_mode == CM_SG && h16 && N <= 64 && K <= 128), "nbp_gemm_bf16: C is null");
  NBP_REQUIRE(K % 8 == 0 && N % 4 == 0 && ldb % 8 == 0, "nbp_gemm_bf16: K, ldb multiples of 8, N of 4 (K=%d N=%d)", K, N);
  NBP_REQUIRE(a_mode >= 0 && a_mode <= 2 && (c_mode == CM_PLAIN || c_mode == CM_D2S || c_mode == CM_SG ||
              c_mode == CM_SGBWD || c_mode == CM_CHANDOT), "nbp_gemm_bf16: mode");
  NBP_REQUIRE(c_mode != CM_CHANDOT || (a_mode == AM_PLAIN && h16 && R && pre && !bias &&
                                       rows_per_img > 0 && rows_per_img % 64 == 0 && M % rows_per_img == 0 &&
                                       N % 8 == 0 && ldc % 8 == 0),
              "nbp_gemm_bf16: channel-dot epilogue needs 16-bit storage, R (g), pre (the slab), rows_per_img a "
              "multiple of 64 dividing M");
  NBP_REQUIRE(c_mode != CM_SG || (pre && N % 2 == 0 && ldc % 2 == 0 && !R),
              "nbp_gemm_bf16: SimpleGate epilogue needs pre (the gate map), even N and ldc, no residual");
  NBP_REQUIRE(c_mode != CM_SGBWD || (R && !bias && !pre && ldc >= 2L * N),
              "nbp_gemm_bf16: SimpleGate-backward epilogue needs R (the interleaved gate input) and ldc >= 2N");
  NBP_REQUIRE(a_mode != AM_SCALE || (a_scale && rows_per_img > 0), "nbp_gemm_bf16: a_scale");
  NBP_REQUIRE((a_mode != AM_S2D && c_mode != CM_D2S) || (gh > 0 && gw > 0 && cs > 0 && cs % 8 == 0),
              "nbp_gemm_bf16: s2d geometry (cs multiple of 8)");
  NBP_REQUIRE(a_mode != AM_S2D || K == 4 * cs, "nbp_gemm_bf16: S2D needs K == 4*cs");
  NBP_REQUIRE(c_mode != CM_D2S || N == 4 * cs, "nbp_gemm_bf16: D2S needs N == 4*cs");
  NBP_REQUIRE(a_mode == AM_S2D || lda % 8 == 0, "nbp_gemm_bf16: lda alignment");
  // the tile dispatch of each 16-bit type lives in its own translation unit (gemm16_bf16.hip / gemm16_fp16.hip):
  // the template instances of one type take minutes to compile, the two compile in parallel
  const int rc = (hd == 2 ? nbp::gemm16_entry_fp16 : nbp::gemm16_entry_bf16)(
      A, lda, a_mode, a_scale, rows_per_img, a_dtype, Bw, ldb, C, ldc, c_mode, c_dtype, M, N, K, gh, gw, cs, bias, R,
      rscale, pre, S(s));
  if (rc == 1) return check_launch("gemm_bf16(skinny)");
  NBP_REQUIRE(C, "nbp_gemm_bf16: C is null and the skinny path does not serve this shape");
  if (rc) return rc;
  return check_launch("gemm_bf16");
}

size_t nbp_dgrad_ln_workspace_floats(long M, int N) {
  return (size_t)2 * (N == 128 || N == 256 || N == 512 ? (M + 63) / 64 : skinny_blocks(M)) * N;
}

int nbp_dgrad_ln_bwd(const void* A, long lda, const void* Wt, long ldb, int M, int N, int K, const void* x,
                     const float* stats, const float* lnw, const void* dres, void* dx, float* dlnw, float* dlnb,
                     float* ws, size_t ws_floats, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(A && Wt && x && stats && lnw && dres && dx && dlnw && dlnb && ws && M > 0, "nbp_dgrad_ln_bwd: bad args");
  NBP_REQUIRE(dtype == 1 || dtype == 2, "nbp_dgrad_ln_bwd: 16-bit storage (dtype 1 bf16 / 2 fp16)");
  float *slab_w, *slab_b;
  long nb;
  if (N == 128 || N == 256 || N == 512) {  // 64 x N tiles of the tiled kernel: a whole row per tile
    NBP_REQUIRE(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "nbp_dgrad_ln_bwd: K, lda, ldb multiples of 8");
    NBP_REQUIRE(N != 512 || (K > 32 && (glds_depth() < 0 || glds_depth() >= 2)), "nbp_dgrad_ln_bwd: N = 512 runs on the LDS-DMA tiles only");
    nb = (M + 63) / 64;
    NBP_REQUIRE(ws_floats >= (size_t)2 * nb * N, "nbp_dgrad_ln_bwd: workspace too small");
    GemmPB p{A, lda, nullptr, 1, Wt, ldb, dx, N, M, N, K, 0, 0, 0, nullptr, x,
             nullptr, nullptr, lnw, nullptr, nullptr, nullptr, 0.f, reinterpret_cast<const float2*>(stats), dres, ws,
             ws + nb * N};
    NBP_DISPATCH_H(dtype, {
      if (N == 512) launch<64, 512, AM_PLAIN, CM_LNBWD, H, H, H>(p, S(s));
      else if (N == 256) launch<64, 256, AM_PLAIN, CM_LNBWD, H, H, H>(p, S(s));
      else launch<64, 128, AM_PLAIN, CM_LNBWD, H, H, H>(p, S(s));
    });
    slab_w = p.slab_w;
    slab_b = p.slab_b;
  } else {
    NBP_REQUIRE((N == 32 || N == 64) && K % 8 == 0 && K <= 128 && lda % 8 == 0 && ldb % 8 == 0,
                "nbp_dgrad_ln_bwd: N must be 32, 64, 128, 256 or 512, K <= 128 (multiple of 8) (N=%d K=%d)", N, K);
    const long nbmax = skinny_blocks(M);  // the slab layout; the launch uses nb <= nbmax of them
    NBP_REQUIRE(ws_floats >= (size_t)2 * nbmax * N, "nbp_dgrad_ln_bwd: workspace too small");
    slab_w = ws;
    slab_b = ws + nbmax * N;
    NBP_DISPATCH_H(dtype, {
      SkinnyP<H> p{reinterpret_cast<const H*>(A), lda, nullptr, 1, reinterpret_cast<const H*>(Wt), ldb,
                   reinterpret_cast<H*>(dx), N, M, N, K, nullptr, reinterpret_cast<const H*>(x), nullptr, nullptr,
                   reinterpret_cast<const float2*>(stats), lnw, reinterpret_cast<const H*>(dres), slab_w, slab_b};
      nb = launch_skinny<AM_PLAIN, CM_LNBWD, H>(p, S(s));
    });
  }
  int rc = check_launch("dgrad_ln_bwd");
  if (rc) return rc;
  rc = nbp_reduce_slab(slab_w, (int)nb, N, dlnw, s);
  if (rc) return rc;
  return nbp_reduce_slab(slab_b, (int)nb, N, dlnb, s);
}

size_t nbp_dgrad_ln_bwd_wg_workspace_floats(long M, int N) {
  return N == 32 ? (size_t)skinny_blocks(M) * (2 * N + 2048 + 64) : 0;
}

int nbp_dgrad_ln_bwd_wg(const void* A, long lda, const void* Wt, long ldb, int M, int N, int K, const void* x,
                        const float* stats, const float* lnw, const float* lnb, const void* dres, void* dx, float* dlnw,
                        float* dlnb, float* dW, float* db, float* ws, size_t ws_floats, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(A && Wt && x && stats && lnw && lnb && dres && dx && dlnw && dlnb && dW && db && ws && M > 0,
              "nbp_dgrad_ln_bwd_wg: bad args");
  NBP_REQUIRE(dtype == 1 || dtype == 2, "nbp_dgrad_ln_bwd_wg: 16-bit storage (dtype 1 bf16 / 2 fp16)");
  NBP_REQUIRE(N == 32 && K == 64 && lda % 8 == 0 && ldb % 8 == 0, "nbp_dgrad_ln_bwd_wg: N = 32, K = 64 (N=%d K=%d)", N, K);
  const long nb = skinny_wg_blocks(M);
  NBP_REQUIRE(ws_floats >= nbp_dgrad_ln_bwd_wg_workspace_floats(M, N), "nbp_dgrad_ln_bwd_wg: workspace too small");
  float* slab_w = ws;
  float* slab_b = slab_w + nb * N;
  float* sw = slab_b + nb * N;
  float* sb = sw + nb * 2048;
  NBP_DISPATCH_H(dtype, {
    SkinnyP<H> p{reinterpret_cast<const H*>(A), lda, nullptr, 1, reinterpret_cast<const H*>(Wt), ldb,
                 reinterpret_cast<H*>(dx), N, M, N, K, nullptr, reinterpret_cast<const H*>(x), nullptr, nullptr,
                 reinterpret_cast<const float2*>(stats), lnw, reinterpret_cast<const H*>(dres), slab_w, slab_b};
    p.lnb_f = lnb;
    p.slab_w2 = sw;
    p.slab_b2 = sb;
    gemm_skinny_kernel<1, 4, AM_PLAIN, CM_LNBWD, H, true><<<dim3((unsigned)nb), 256, 0, S(s)>>>(p);
  });
  int rc = check_launch("dgrad_ln_bwd_wg");
  if (rc) return rc;
  if ((rc = nbp_reduce_slab(slab_w, (int)nb, N, dlnw, s))) return rc;
  if ((rc = nbp_reduce_slab(slab_b, (int)nb, N, dlnb, s))) return rc;
  if ((rc = nbp_reduce_slab(sw, (int)nb, 2L * N * N, dW, s))) return rc;
  return nbp_reduce_slab(sb, (int)nb, 2L * N, db, s);
}

int nbp_gemm_res_ln(const void* A, long lda, int a_mode, const float* a_scale, int rows_per_img, const void* Bw,
                    long ldb, void* C, int M, int N, int K, const float* bias, const void* R, const float* rscale,
                    const float* lnw, const float* lnb, void* nout, float* stats, float eps, int dtype,
                    nbp_stream_t s) {
  NBP_REQUIRE(A && Bw && C && R && lnw && lnb && nout && stats && M > 0, "nbp_gemm_res_ln: bad args (R: the residual)");
  NBP_REQUIRE(dtype == 1 || dtype == 2, "nbp_gemm_res_ln: 16-bit storage (dtype 1 bf16 / 2 fp16)");
  NBP_REQUIRE(a_mode == AM_PLAIN || (a_mode == AM_SCALE && a_scale && rows_per_img > 0), "nbp_gemm_res_ln: a_mode");
  if (N == 128 || N == 256 || N == 512) {  // 64 x N tiles of the tiled kernel: a whole row per tile
    NBP_REQUIRE(K % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0, "nbp_gemm_res_ln: K, lda, ldb multiples of 8");
    NBP_REQUIRE(N != 512 || (K > 32 && (glds_depth() < 0 || glds_depth() >= 2)), "nbp_gemm_res_ln: N = 512 runs on the LDS-DMA tiles only");
    GemmPB p{A, lda, a_scale, rows_per_img, Bw, ldb, C, N, M, N, K, 0, 0, 0, bias,
             R, rscale, nullptr, lnw, lnb, nout, reinterpret_cast<float2*>(stats), eps};
    NBP_DISPATCH_H(dtype, {
      if (N == 512 && a_mode == AM_SCALE) launch<64, 512, AM_SCALE, CM_RESLN, H, H, H>(p, S(s));
      else if (N == 512) launch<64, 512, AM_PLAIN, CM_RESLN, H, H, H>(p, S(s));
      else if (N == 256 && a_mode == AM_SCALE) launch<64, 256, AM_SCALE, CM_RESLN, H, H, H>(p, S(s));
      else if (N == 256) launch<64, 256, AM_PLAIN, CM_RESLN, H, H, H>(p, S(s));
      else if (a_mode == AM_SCALE) launch<64, 128, AM_SCALE, CM_RESLN, H, H, H>(p, S(s));
      else launch<64, 128, AM_PLAIN, CM_RESLN, H, H, H>(p, S(s));
    });
    return check_launch("gemm_res_ln(tiled)");
  }
  NBP_REQUIRE((N == 32 || N == 64) && K % 8 == 0 && K <= 128 && lda % 8 == 0 && ldb % 8 == 0,
              "nbp_gemm_res_ln: N must be 32, 64, 128, 256 or 512, K <= 128 (multiple of 8) (N=%d K=%d)", N, K);
  NBP_DISPATCH_H(dtype, {
    SkinnyP<H> p{reinterpret_cast<const H*>(A), lda, a_scale, rows_per_img, reinterpret_cast<const H*>(Bw), ldb,
                 reinterpret_cast<H*>(C), N, M, N, K, bias, reinterpret_cast<const H*>(R), rscale, nullptr,
                 nullptr, lnw, nullptr, nullptr, nullptr, lnb, reinterpret_cast<H*>(nout),
                 reinterpret_cast<float2*>(stats), eps};
    if (a_mode == AM_SCALE) launch_skinny<AM_SCALE, CM_RESLN, H>(p, S(s));
    else launch_skinny<AM_PLAIN, CM_RESLN, H>(p, S(s));
  });
  return check_launch("gemm_res_ln");
}

int nbp_gemm_ffn(const void* n2, const void* W4, const float* b4, const void* W5, const float* b5, const void* y,
                 const float* gamma, const float* lnw, const float* lnb, void* out, void* nout, float* stats, int M,
                 int C, float eps, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(n2 && W4 && b4 && W5 && b5 && y && gamma && out && M > 0, "nbp_gemm_ffn: bad args");
  NBP_REQUIRE(!nout || (lnw && lnb && stats), "nbp_gemm_ffn: the next LayerNorm needs lnw, lnb, stats");
  NBP_REQUIRE(dtype == 1 || dtype == 2, "nbp_gemm_ffn: 16-bit storage (dtype 1 bf16 / 2 fp16)");
  NBP_REQUIRE(C == 32, "nbp_gemm_ffn: the fused FFN half serves C = 32 (C=%d)", C);
  NBP_DISPATCH_H(dtype, {
    SkinnyP<H> p{reinterpret_cast<const H*>(n2), C, nullptr, 1, reinterpret_cast<const H*>(W5), C,
                 reinterpret_cast<H*>(out), C, M, C, C, b5, reinterpret_cast<const H*>(y), gamma, nullptr,
                 nullptr, lnw, nullptr, nullptr, nullptr, lnb, reinterpret_cast<H*>(nout),
                 reinterpret_cast<float2*>(stats), eps, nullptr, reinterpret_cast<const H*>(W4), b4};
    gemm_skinny_kernel<1, 2, AM_PLAIN, CM_FFN, H>
        <<<dim3((unsigned)skinny_grid<1, 2, AM_PLAIN, CM_FFN, H>(M)), 256, 0, S(s)>>>(p);
  });
  return check_launch("gemm_ffn");
}

int nbp_dgrad_sg_rc(const void* A, long lda, const void* Wt, long ldb, const void* A2, const void* W2, const float* b2,
                    void* C, int M, int N, int K, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(A && Wt && A2 && W2 && b2 && C && M > 0, "nbp_dgrad_sg_rc: bad args");
  NBP_REQUIRE(dtype == 1 || dtype == 2, "nbp_dgrad_sg_rc: 16-bit storage (dtype 1 bf16 / 2 fp16)");
  NBP_REQUIRE(N == 32 && K == 32 && lda % 8 == 0 && ldb % 8 == 0,
              "nbp_dgrad_sg_rc: N = K = 32 (N=%d K=%d)", N, K);
  NBP_DISPATCH_H(dtype, {
    SkinnyP<H> p{reinterpret_cast<const H*>(A), lda, nullptr, 1, reinterpret_cast<const H*>(Wt), ldb,
                 reinterpret_cast<H*>(C), 2L * N, M, N, K, nullptr, nullptr, nullptr, nullptr,
                 nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f,
                 reinterpret_cast<const H*>(A2), reinterpret_cast<const H*>(W2), b2};
    gemm_skinny_kernel<1, 2, AM_PLAIN, CM_SGBWD_RC, H>
        <<<dim3((unsigned)skinny_grid<1, 2, AM_PLAIN, CM_SGBWD_RC, H>(M)), 256, 0, S(s)>>>(p);
  });
  return check_launch("dgrad_sg_rc");
}

size_t nbp_dgrad_sg_rc_wg_workspace_floats(long M, int N) {
  return N == 32 ? (size_t)skinny_blocks(M) * (2048 + 1024 + 64 + 32) : 0;
}

int nbp_dgrad_sg_rc_wg(const void* A, long lda, const void* Wt, long ldb, const void* A2, const void* W2,
                       const float* b2, void* C, int M, int N, int K, float* U, float* V, float* dW2, float* db2,
                       float* ws, size_t ws_floats, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(A && Wt && A2 && W2 && b2 && C && U && V && dW2 && db2 && ws && M > 0,
              "nbp_dgrad_sg_rc_wg: bad args");
  NBP_REQUIRE(dtype == 1 || dtype == 2, "nbp_dgrad_sg_rc_wg: 16-bit storage (dtype 1 bf16 / 2 fp16)");
  NBP_REQUIRE(N == 32 && K == 32 && lda % 8 == 0 && ldb % 8 == 0, "nbp_dgrad_sg_rc_wg: N = K = 32 (N=%d K=%d)", N, K);
  const long nb = skinny_wg_blocks(M);
  NBP_REQUIRE(ws_floats >= nbp_dgrad_sg_rc_wg_workspace_floats(M, N), "nbp_dgrad_sg_rc_wg: workspace too small");
  float* sw2 = ws;
  float* su = sw2 + nb * 2048;
  float* sb2 = su + nb * 1024;
  float* sv = sb2 + nb * 64;
  NBP_DISPATCH_H(dtype, {
    SkinnyP<H> p{reinterpret_cast<const H*>(A), lda, nullptr, 1, reinterpret_cast<const H*>(Wt), ldb,
                 reinterpret_cast<H*>(C), 2L * N, M, N, K, nullptr, nullptr, nullptr, nullptr,
                 nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f,
                 reinterpret_cast<const H*>(A2), reinterpret_cast<const H*>(W2), b2, su, sv, sw2, sb2};
    gemm_skinny_kernel<1, 2, AM_PLAIN, CM_SGBWD_RC, H, true><<<dim3((unsigned)nb), 256, 0, S(s)>>>(p);
  });
  int rc = check_launch("dgrad_sg_rc_wg");
  if (rc) return rc;
  // the block partials reduce with the stage's deferred reductions (nbp_wgrad_f32's semantics)
  if ((rc = nbp_reduce_slab(sw2, (int)nb, 2L * N * K, dW2, s))) return rc;
  if ((rc = nbp_reduce_slab(sb2, (int)nb, 2L * N, db2, s))) return rc;
  if ((rc = nbp_reduce_slab(su, (int)nb, (long)N * N, U, s))) return rc;
  return nbp_reduce_slab(sv, (int)nb, N, V, s);
}

int nbp_weights_bf16(const float* flat, long n, void* out, const long* desc, int ndesc, void* out_t, int dtype,
                     nbp_stream_t s) {
  NBP_REQUIRE(flat && out && n > 0 && (ndesc == 0 || (desc && out_t)) && ndesc <= 65535, "nbp_weights_bf16: bad args");
  NBP_REQUIRE(dtype == 1 || dtype == 2, "nbp_weights_bf16: dtype 1 (bf16) or 2 (fp16)");
  NBP_REQUIRE((((uintptr_t)flat | (uintptr_t)out) & 15) == 0 && (ndesc == 0 || ((uintptr_t)out_t & 15) == 0),
              "nbp_weights_bf16: flat / out / out_t must be 16-byte aligned (vector loads and stores)");
  long g = (n / 8 + 255) / 256;
  NBP_DISPATCH_H(dtype, {
    cvt_bf16_kernel<H><<<(int)(g > 4096 ? 4096 : (g < 1 ? 1 : g)), 256, 0, S(s)>>>(flat, n, reinterpret_cast<H*>(out));
    // 64 tile-strided workgroups per matrix: the largest GEMM weight (1024 x 512) has 128 tiles
    if (ndesc > 0)
      transpose_bf16_kernel<H><<<dim3(64, ndesc), 256, 0, S(s)>>>(flat, desc, reinterpret_cast<H*>(out_t));
  });
  return check_launch("weights_bf16");
}

}  // extern "C"
