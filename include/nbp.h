/*
 * nbp.h — C-ABI of the MI355X (gfx950) NewBP-NAFNet hot-path library  (liblowlight_nbp.so).
 *
 * The reference (RUA1027/Lowlight_Image_Enhancement) is pure Python; its "operator boundary" is the set of
 * torch ops its hot-path modules call.  Each entry point below replaces the reference op named in its comment
 * (file:line relative to the reference root).  The Python host layer (lowlight_image_enhancement_amd/) binds
 * these with ctypes and keeps the reference's module/function names.
 *
 * Conventions
 *  - All tensors are caller-owned device pointers (fp32 unless stated).  The library never allocates
 *    persistent device memory: scratch is a caller-provided workspace sized by the *_workspace_* queries.
 *  - Every call is asynchronous on the caller's stream (hipStream_t passed as nbp_stream_t) and stateless.
 *  - Return 0 on success or a negative NBP_ERR_* code; nbp_last_error_string() describes the last failure
 *    (thread-local).
 *  - Activations inside the network are NHWC ([B][H][W][C], M = B*H*W rows of C channels); images at the
 *    network boundary and the loss terms are NCHW, the reference's public layout.
 *  - Scalars produced on the device (losses, norms) are written to device memory; gradients of scalar losses
 *    read the upstream gradient from device memory (`up`), so nothing forces a host sync.
 *  - `dtype` selects the storage of NHWC activations/activation-gradients: 0 fp32, 1 bf16, 2 fp16 (the 16-bit perf
 *    modes; fp16 is the reference's autocast dtype).  16-bit storage means 16-bit MFMA operands of the same type.
 *    Math, statistics, parameters and parameter gradients are fp32 in every mode.
 */
#ifndef NBP_H_
#define NBP_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NBP_VERSION 1
typedef void* nbp_stream_t; /* hipStream_t */

enum { NBP_OK = 0, NBP_ERR_ARG = -1, NBP_ERR_LAUNCH = -2, NBP_ERR_INTERNAL = -3 };

const char* nbp_last_error_string(void);
int nbp_version(void);

/* ------------------------------------------------------------------ physics branch (NewBP) */
/* CrosstalkPSF.__init__ normalisation k / clamp_min(k.sum(1), 1e-12) (NewBP_model/newbp_layer.py:102-106),
 * host-side, bit-exact with torch's CPU fp32 row sum (8 interleaved accumulators). */
int nbp_psf_normalize_host(const float* k, int n_kernels, int len, float* out);
/* depthwise KxK conv on NCHW, pad_mode 0 zeros / 1 replicate / 2 reflect; k [C][KH*KW] or shared [1][KH*KW]:
 * CrosstalkPSF.forward F.conv2d(x, K, padding=1, groups=3) (newbp_layer.py:109-126); pre_clamp applies
 * clamp(0,1) to the input first. */
int nbp_dwconv_nchw_fwd(const float* x, const float* k, int k_shared, float* y, int N, int C, int H, int W, int KH,
                        int KW, int pad_mode, int pre_clamp, nbp_stream_t s);
/* adjoint of the zero-padded depthwise conv = conv_transpose2d(g, K, padding=1, groups=3)
 * (core_tests/test_physics_loss_grad.py:65-86). */
int nbp_dwconv_nchw_bwd_zero(const float* gy, const float* k, int k_shared, float* gx, int N, int C, int H, int W,
                             int KH, int KW, nbp_stream_t s);
/* Fused physics L1: loss = mean |PSF_pad(clamp?(bhat)) - clamp?(clamp?(a) * ratio)|
 *   pad_mode 0 + normalised K + clamp_align : PhysicalConsistencyLossSRGB (NewBP_model/losses.py:206-220) with
 *     align_exposure_srgb (:195-203);
 *   pad_mode 1 (replicate) + raw K           : PhysicsConsistencyLoss (losses.py:158-192).
 * ratio: [N*C] per (sample, channel) (ratio_full = 0) or a full [N,C,H,W] map.  sign_map (optional, [N,C,H,W])
 * keeps sign(residual) for the backward.  ws: nbp_phys_l1_workspace_doubles() doubles. */
size_t nbp_phys_l1_workspace_doubles(int N, int C, int H, int W);
int nbp_phys_l1_fwd(const float* bhat, const float* a, const float* ratio, int ratio_full, const float* k, int k_shared,
                    int N, int C, int H, int W, int KH, int KW, int pad_mode, int clamp_bhat, int clamp_a_in,
                    int clamp_align, double* ws, float* loss, float* sign_map, nbp_stream_t s);
/* d loss / d bhat = up[0]/numel * PSF^T(sign) (* 1[0 <= bhat <= 1] when clamp_bhat). */
int nbp_phys_l1_bwd(const float* sign_map, const float* bhat, const float* k, int k_shared, const float* up, int N,
                    int C, int H, int W, int KH, int KW, int pad_mode, int clamp_bhat, float* gx, nbp_stream_t s);
/* PhysicsConsistencyLoss, groups == 1 branch (NewBP_model/losses.py:182-191: a [Co,1,kh,kw] kernel with Co not in
 * {1, C} expanded to [Co,C,kh,kw], or a full [Co,C,kh,kw] kernel): yhat = conv2d(ReplicationPad(bhat), k) [N,Co,H,W]
 * against al = clamp?(a * ratio) [N,Ca,H,W] (ratio [N*Ca] or full), L1 mean over torch's channel broadcast
 * Cb = max(Co, Ca) (Co == Ca, or one of them 1).  k: [Co][C][KH][KW] (the expansion done by the caller).
 * ws: nbp_phys_l1_workspace_doubles(N, Cb, H, W); sign_map [N][Cb][H][W] for the backward. */
int nbp_phys_full_fwd(const float* bhat, const float* a, const float* ratio, int ratio_full, const float* k, int N,
                      int C, int Co, int Ca, int H, int W, int KH, int KW, int clamp_align, double* ws, float* loss,
                      float* sign_map, nbp_stream_t s);
/* d loss / d bhat = up[0] / (N*Cb*H*W) * (replicate-pad adjoint of conv2d)^T(sign). */
int nbp_phys_full_bwd(const float* sign_map, const float* k, const float* up, int N, int C, int Co, int Ca, int H, int W,
                      int KH, int KW, float* gx, nbp_stream_t s);
/* Gradient w.r.t. the short exposure A of either physics L1 (the reference's modules are plain autograd, so A gets one):
   ga = -up[0] / (N*Cb*H*W) * sum_{cb -> ca} sign_map * ratio * clamp masks (clamp_align: of a*ratio, clamp_a_in: of a),
   sign_map [N][Cb][H][W] from the forward; Ca == Cb (depthwise losses) or Ca == 1 (broadcast). */
int nbp_phys_a_bwd(const float* sign_map, const float* a, const float* ratio, int ratio_full, int N, int Ca, int Cb, int H,
                   int W, int clamp_a_in, int clamp_align, const float* up, float* ga, nbp_stream_t s);
/* _phys_cons_core (metrics/phys_consistency.py:193-255) for phys_cons_raw (:260) / phys_cons_srgb (:323):
 * full [Co][Ci][KH][KW] PSF (already prepared), pad 0/1/2, ratio_mode 0 [N] / 1 [N,1,H,W] / 2 [N,Co,H,W],
 * crop 'valid' (crop_valid=1) or 'same', clamp01 of the synthesised observation (sRGB), L1 or Charbonnier
 * sqrt(d^2 + eps^2).  out[0..N-1] per-sample means, out[N] batch mean, out[N+1] batch sum;
 * amap (optional) = |y - obs| over the compared region, [N][Co][Ho][Wo]. */
size_t nbp_phys_cons_workspace_doubles(int N, int H, int W);
int nbp_phys_cons(const float* pred, const float* obs, const float* psf, const float* ratio, int ratio_mode, int N,
                  int Ci, int Co, int H, int W, int KH, int KW, int pad_mode, int crop_valid, int clamp01_out,
                  int charbonnier, float eps, float* amap, double* ws, float* out, nbp_stream_t s);
/* align_exposure_srgb (NewBP_model/losses.py:195-203): clamp(a * ratio, 0, 1), ratio [N*C] or full [N,C,H,W]. */
int nbp_align_exposure(const float* a, const float* ratio, int ratio_full, float* out, int N, int C, long HW,
                       nbp_stream_t s);
/* torch.isfinite(x).all() (phys_consistency.py:58-61, losses.py:298-306): *flag_dev = 1 if any non-finite. */
int nbp_all_finite(const float* x, long n, int* flag_dev, nbp_stream_t s);

/* ------------------------------------------------------------------ NAFNet (NHWC) */
/* 1x1 conv / channel contraction on MFMA (fp32 in, fp32 accumulate):  C = A(M,K) . B + epilogue
 *   NAFBlock conv1/conv3/conv4/conv5 (NAFNet_arch.py:31-48), down conv 2x2/s2 (:106-108) through a_mode 1
 *   (space-to-depth gather), up conv 1x1 + PixelShuffle(2) + skip add (:117-122,148-149) through c_mode 1
 *   (depth-to-space scatter + residual), and the dgrad of all of them.
 *   a_mode: 0 plain A[m*lda+k], 1 S2D gather of a 2x map (K = 4*cs), 2 per-image column scale (SCA, :67)
 *   b_nk  : 1 B stored [N][K] (conv weight [out][in]); 0 B stored [K][N]
 *   c_mode: 0 plain C[m*ldc+n], 1 D2S scatter into a 2x map (N = 4*cs)
 *   epilogue: v = acc + bias[n]; pre (opt) = v; C = R ? R + rscale[n] * v : v   (layer-scale residual :72,80) */
int nbp_gemm_f32(const float* A, long lda, int a_mode, const float* a_scale, int rows_per_img, const float* B,
                 long ldb, int b_nk, float* C, long ldc, int c_mode, int M, int N, int K, int gh, int gw, int cs,
                 const float* bias, const float* R, const float* rscale, float* pre, nbp_stream_t s);
/* 16-bit-operand MFMA variant (perf modes; AMP-equivalent operands, fp32 accumulate): C = A . Bw^T, Bw 16-bit
 * [N][ldb]; a_dtype / c_dtype: 0 fp32, 1 bf16, 2 fp16 storage of A and of C/R/pre (16-bit ones agree).  The operand
 * type (Bw, 16-bit A / C) is fp16 when either side is fp16, else bf16 (so fp32 A and C take bf16 weights).  Same a_mode/c_mode/epilogue as nbp_gemm_f32;
 * dgrads pass the transposed weight copy.  K, ldb multiples of 8; S2D/D2S need cs % 8 == 0.  Extra c_modes fusing
 * SimpleGate (NAFNet_arch.py:22-25,75-76) on interleaved channel pairs: 4 = forward (C = t, pre <- g[M][N/2] with
 * g[c] = t[2c] * t[2c+1]), 5 = backward (acc = dg[M][N]; R = t [M][2N] interleaved; C[2c] = dg[c] * t[2c+1],
 * C[2c+1] = dg[c] * t[2c], row stride ldc). */
int nbp_gemm_bf16(const void* A, long lda, int a_mode, const float* a_scale, int rows_per_img, int a_dtype,
                  const void* Bw, long ldb, void* C, long ldc, int c_mode, int c_dtype, int M, int N, int K, int gh,
                  int gw, int cs, const float* bias, const void* R, const float* rscale, void* pre, nbp_stream_t s);
/* 1x1-conv input gradient fused with the LayerNorm2d backward that follows it (bf16; NAFBlock conv4 -> norm2 and
 * conv1 -> norm1 at N = C in {32, 64}, NAFNet_arch.py:60-80 + arch_util.py:277-289):
 *   dn = A[M,K] . Wt[N,K]^T (never stored),  dx = (g - yhat*mean(g*yhat) - mean(g)) / den + dres,  g = dn * lnw,
 *   yhat = (x - mu) / den from stats = (mu, den) per row;  dlnw = sum dn*yhat, dlnb = sum dn (slab reductions into
 *   ws, deferred like nbp_wgrad_f32's).  ws: nbp_dgrad_ln_workspace_floats(M, N). */
size_t nbp_dgrad_ln_workspace_floats(long M, int N);
int nbp_dgrad_ln_bwd(const void* A, long lda, const void* Wt, long ldb, int M, int N, int K, const void* x,
                     const float* stats, const float* lnw, const void* dres, void* dx, float* dlnw, float* dlnb,
                     float* ws, size_t ws_floats, int dtype, nbp_stream_t s);
/* nbp_dgrad_ln_bwd plus conv1's weight gradient from the same tiles (level 0: N = C = 32, K = 2C = 64; the separate
 * nbp_wgrad_f32 launch and its re-read of dt / n1 disappear): dW = A^T n1 [K][N], db = colsum A [K], with n1 = lnw yhat
 * + lnb rebuilt from x / stats exactly as nbp_ln_fwd_nhwc (and the nbp_gemm_res_ln / nbp_gemm_ffn epilogues) stored
 * it.  Block partials in ws (nbp_dgrad_ln_bwd_wg_workspace_floats), reduced like nbp_wgrad_f32's slabs (deferred with
 * the stage).  dx, dlnw, dlnb as nbp_dgrad_ln_bwd (dx bit for bit).  Reference: NAFNet_arch.py:60-64 (norm1 -> conv1),
 * whose conv1 weight gradient torch autograd computes in a separate pass. */
size_t nbp_dgrad_ln_bwd_wg_workspace_floats(long M, int N);
int nbp_dgrad_ln_bwd_wg(const void* A, long lda, const void* Wt, long ldb, int M, int N, int K, const void* x,
                        const float* stats, const float* lnw, const float* lnb, const void* dres, void* dx, float* dlnw,
                        float* dlnb, float* dW, float* db, float* ws, size_t ws_floats, int dtype, nbp_stream_t s);
/* NAFBlock conv3 / conv5 (N = C in {32, 64} on the skinny kernel with K <= 128, or 128 on 64 x 128 tiles; bf16) with
 * the next LayerNorm2d forward in the epilogue:
 * C = R + rscale * (A W^T + bias) (the block's y / out, NAFNet_arch.py:70-78) and nout / stats = LN(C) exactly as
 * nbp_ln_fwd_nhwc computes them from the stored C (arch_util.py:266-275); C, nout row stride N. */
int nbp_gemm_res_ln(const void* A, long lda, int a_mode, const float* a_scale, int rows_per_img, const void* Bw,
                    long ldb, void* C, int M, int N, int K, const float* bias, const void* R, const float* rscale,
                    const float* lnw, const float* lnb, void* nout, float* stats, float eps, int dtype,
                    nbp_stream_t s);
/* The level-0 NAFBlock FFN half in one pass (NAFNet_arch.py:74-80; C = 32): out = y + gamma (.) (SG(n2 W4^T + b4)
 * W5^T + b5) and, when nout is given, the next block's LayerNorm2d of out into nout / stats (as nbp_gemm_res_ln).  W4 /
 * b4: conv4's bf16 weight and bias with the SimpleGate pairs interleaved (2C rows), W5: conv5's [C][C].  The gate map
 * g2 = SG(t4) is formed in registers and never stored (the level-0 backward rebuilds it, nbp_dgrad_sg_rc_wg); out is
 * bitwise the two-launch form's (nbp_gemm_bf16 CM_SG, then nbp_gemm_res_ln / CM_PLAIN with the residual). */
int nbp_gemm_ffn(const void* n2, const void* W4, const float* b4, const void* W5, const float* b5, const void* y,
                 const float* gamma, const float* lnw, const float* lnb, void* out, void* nout, float* stats, int M,
                 int C, float eps, int dtype, nbp_stream_t s);
/* The deep-level NAFBlock FFN half in ONE row-stationary launch (NAFNet_arch.py:69-80 after the SCA; C 128 / 256 / 512,
 * 16-bit): y = x + beta (.) ((g (.) a) W3^T + b3); n2 / st2 = LayerNorm2d(y) (norm2); t4 = n2 W4^T + b4 (SimpleGate pairs
 * interleaved, 2C columns); g2 = t4[2c] t4[2c + 1]; out = y + gamma (.) (g2 W5^T + b5); with lnw1 / lnb1 also the next
 * block's norm1 of out into nn1 / nst1.  a: [B][C] SCA scale (per image of rows_per_img rows); weights w3 / w4 / w5:
 * 16-bit copies in fragment order (nbp_frag16).  Replaces nbp_gemm_bf16 / nbp_gemm_res_ln (conv3) + nbp_ln_fwd_nhwc + nbp_gemm_bf16 CM_SG
 * (conv4) + nbp_gemm_res_ln / nbp_gemm_bf16 (conv5) + nbp_ln_fwd_nhwc, bitwise: every stored tensor equals theirs.
 * Stats are (mu, den) float pairs.  nbp_ffn_rows_supported(M, C, rows_per_img, dtype): 1 for the shapes served
 * (rows_per_img a multiple of 32). */
int nbp_ffn_rows_supported(int M, int C, int rows_per_img, int dtype);
/* 16-bit matrices [N][K] at their flat offsets (desc = [ndesc][3] int64 {offset, N, K}; N a multiple of 32, K of 16)
 * copied into fragment order at the same offsets of out: 1-KB blocks (32-row tile nt, 16-wide k-step ks) in (nt, ks)
 * order, lane l's 16 bytes = row 32 nt + (l & 31), k 16 ks + 8 (l >> 5) .. + 7 (the 32 x 32 x 16 MFMA B operand of
 * nbp_ffn_rows_fwd / nbp_ffn_rows_bwd; one contiguous load per wave).  A permutation: values bitwise the source's. */
int nbp_frag16(const void* src, const long* desc, int ndesc, void* out, nbp_stream_t s);
/* The backward of nbp_ffn_rows_fwd's chain in ONE row-stationary launch (levels C 128 / 256 / 512, 16-bit): dg2 = dout
 * W5'^T, dt4 = SimpleGate backward on the stored t4, dn2 = dt4 W4^T, dy = LayerNorm2d backward (norm2: y, st2, lnw2) +
 * dout, dh = dy W3'^T, where W5' / W3' are the layer-scale-folded transposed weights of the tiled dgrads (gamma / beta
 * (.) W)^T and all three weights are fragment-ordered (nbp_frag16 of the transposed 16-bit copies); plus, per 32-row
 * block b, slab_w[b] = sum dn2 * yhat, slab_b[b] = sum dn2 (norm2's weight / bias gradient partials) and da[b] = sum dh
 * (.) g (the SCA channel-dot partials, [B][rows_per_img / 32][C]).  Replaces nbp_gemm_bf16 CM_SGBWD + nbp_dgrad_ln_bwd
 * (or nbp_gemm_bf16 + nbp_ln_bwd_nhwc at C 512) + nbp_gemm_bf16 CM_CHANDOT: dt4 / dy / dh bitwise theirs, the partial
 * sums up to fp32 summation order.  With dt1 (dout null): first the FOLLOWING block's conv1 input gradient + norm1 backward
 * (the executor's pending one; both blocks of one level, NAFNet_arch.py:60-63 backward): dx1 = LayerNorm2d backward(dt1
 * W1^T; x1, st1, lnw1) + dres1 (that block's dy), stored and taken as this block's dout, with norm1's partials per 32-row
 * block in slab_w1 / slab_b1 (w1t: fragment-ordered W1^T [C][2C]; dx1 bitwise nbp_dgrad_ln_bwd / nbp_gemm_bf16 +
 * nbp_ln_bwd_nhwc).  Shapes as nbp_ffn_rows_supported. */
int nbp_ffn_rows_bwd(const void* dout, const void* t4, const void* y, const float* st2, const float* lnw2, const void* g,
                     const void* w5t, const void* w4t, const void* w3t, void* dt4, void* dy, void* dh, float* slab_w,
                     float* slab_b, float* da, const void* dt1, const void* w1t, const void* x1, const float* st1,
                     const float* lnw1, const void* dres1, void* dx1, float* slab_w1, float* slab_b1, int M, int C,
                     int rows_per_img, int dtype, nbp_stream_t s);
int nbp_ffn_rows_fwd(const void* g, const float* a, int rows_per_img, const void* x, const void* w3, const float* b3,
                     const float* beta, const float* lnw2, const float* lnb2, const void* w4, const float* b4,
                     const void* w5, const float* b5, const float* gamma, const float* lnw1, const float* lnb1, void* y,
                     void* n2, float* st2, void* t4, void* g2, void* out, void* nn1, float* nst1, int M, int C,
                     float eps, int dtype, nbp_stream_t s);
/* conv5 input gradient + SimpleGate backward with the gate input recomputed (bf16, N = K = C = 32: level 0, whose conv4
 * forward runs on the same skinny MFMA sequence): dg = A . Wt^T (the conv5 dgrad), t = A2 . W2^T + b2 rebuilt per tile (the conv4 forward: A2 = its input n2 [M][K],
 * W2 [2N][K] bf16 with SimpleGate pairs interleaved, b2 fp32), C[m][2c] = dg[c] t[2c+1], C[m][2c+1] = dg[c] t[2c]
 * (NAFNet_arch.py:22-25, 76-78); equals CM_SGBWD on the stored t bit for bit.  The forward then skips storing t
 * (nbp_gemm_bf16 CM_SG with C = NULL). */
int nbp_dgrad_sg_rc(const void* A, long lda, const void* Wt, long ldb, const void* A2, const void* W2, const float* b2,
                    void* C, int M, int N, int K, int dtype, nbp_stream_t s);
/* nbp_dgrad_sg_rc plus the weight gradients that read the same operands (level 0: the reads of the separate
 * nbp_wgrad_f32 launches for conv5's U / V and conv4's weight / bias disappear): U = A^T g [N][N] with g the SimpleGate
 * output rebuilt from t (the forward's stored g, bit for bit), V = colsum A [N], dW2 = C^T A2 [2N][K] (C = the stored
 * dt), db2 = colsum C [2N]; block partials in ws (nbp_dgrad_sg_rc_wg_workspace_floats), reduced like nbp_wgrad_f32's
 * slabs (deferred with the stage).  N = K = 32.  Reference: NAFNet_arch.py:76-80 (conv4 / SimpleGate / conv5),
 * whose weight gradients torch autograd computes in separate passes. */
size_t nbp_dgrad_sg_rc_wg_workspace_floats(long M, int N);
int nbp_dgrad_sg_rc_wg(const void* A, long lda, const void* Wt, long ldb, const void* A2, const void* W2,
                       const float* b2, void* C, int M, int N, int K, float* U, float* V, float* dW2, float* db2,
                       float* ws, size_t ws_floats, int dtype, nbp_stream_t s);
/* per-step weight prep: out = h(flat); for each desc {offset, rows, cols, scale_offset} (int64, device)
 * out_t[offset..] = h(diag(s) . flat matrix)^T, h = bf16 (dtype 1) or fp16 (dtype 2), with s = flat[scale_offset..] (rows values), or no scaling when
 * scale_offset < 0 (the NAFBlock layer scales folded into the conv3 / conv5 dgrad operands). */
int nbp_weights_bf16(const float* flat, long n, void* out, const long* desc, int ndesc, void* out_t, int dtype,
                     nbp_stream_t s);
/* weight gradient dW[n][k] = sum_m G(m,n) X(m,k) (+ db[n] = sum_m G(m,n)): split over M, fixed-order slab reduce. */
size_t nbp_wgrad_workspace_floats(int M, int N, int K);
/* Grouping: between nbp_wgrad_group(1, s) and nbp_wgrad_group(0, s) the wide plain bf16 weight gradients
 * (N, K multiples of 128, G and X row-major) issued on this thread are queued and launched together by the end call
 * (one launch, each problem's tiles and results unchanged); the other forms launch at once.  The callers' slab
 * reductions are queued as usual. */
int nbp_wgrad_group(int begin, nbp_stream_t s);
int nbp_wgrad_f32(const void* G, long ldg, int g_mode, const void* X, long ldx, int x_mode, const float* x_scale,
                  int rows_per_img, int M, int N, int K, int gh, int gw, int cs_g, int cs_x, float* dW, float* db,
                  float* ws, size_t ws_floats, int dtype, nbp_stream_t s);
/* out[i] = sum_{s<S} slab[s*L + i] (fixed order); batched: out[b][i] = scale * sum_s slab[b][s][i]. */
int nbp_reduce_slab(const float* slab, int S, long L, float* out, nbp_stream_t s);
/* Deferred gradient reductions (thread-local): after nbp_grad_reduce_defer(s), scale-1 gradient-slab reductions
   issued by this thread (nbp_reduce_slab and the internal ones of nbp_wgrad_f32 / nbp_dw_bwd / nbp_sca_sg_dw_bwd /
   intro / ending / LN backward, on s or on a side stream) are queued; nbp_grad_reduce_flush(stop, s) executes the
   queue on s with one launch per 48 slabs (bitwise identical to immediate mode) and, if stop, ends deferral.  The
   caller orders s after every stream that produced a queued slab and keeps the slabs alive until the flush. */
int nbp_grad_reduce_defer(nbp_stream_t s);
/* Layer-scale residual y = x + s * (h W^T + b) (NAFNet_arch.py:72,80) gradients from U = dy^T h [N][K] and
   V = colsum(dy) [N] of the UNSCALED dy: dW = s (.) U (row-wise), db = s (.) V, ds = rowsum(W (.) U) + b (.) V.
   Queued behind the reductions while deferral is on for s (U/V may then be deferred reduction outputs). */
int nbp_layer_scale_grad(const float* U, const float* V, const float* W, const float* b, const float* scale, float* dW,
                         float* db, float* dscale, int N, int K, nbp_stream_t s);
int nbp_grad_reduce_flush(int stop, nbp_stream_t s);
/* Measurement record of this thread's last call of a kind (host bookkeeping only, no GPU work; bench.py's per-launch
 * roofline accounting).  which = 0: the last nbp_wgrad_f32 -> {queued into the open group (1) or
 * launched (0), M-splits, fp32 slab bytes written, FLOPs 2MNK}; 1: the last nbp_grad_reduce_flush -> {slabs reduced,
 * slab bytes read, bytes written, reduce_multi_kernel (+ post-op) launches}; 2: the last nbp_wgrad_group(0) -> {problems,
 * FLOPs, operand bytes read once, fp32 dW / db bytes, fp32 slab bytes written at the group's M-splits, launches}.
 * Copies min(n, record length) values to out (the rest zero). */
int nbp_last_call_stats(int which, double* out, int n);
/* Per-launch timing of the entries that issue several kernel instances in one call (nbp_wgrad_group, the gradient-
 * reduction flush): nbp_launch_timing(1) clears the record and brackets each such launch of this thread with HIP
 * events (0: off, the default); nbp_launch_timing_get(i, name, cap, out) waits for record i and returns its kernel
 * instance name and out = {milliseconds, algorithmic FLOPs, algorithmic bytes}.  Measurement plumbing of bench.py's
 * per-instance roofline (the reference has no counterpart). */
int nbp_launch_timing(int on);
int nbp_launch_timing_count(void);
int nbp_launch_timing_get(int i, char* name, int cap, double* out);
int nbp_reduce_slab_batched(const float* slab, int batch, int S, long L, float scale, float* out, nbp_stream_t s);

/* LayerNorm2d / LayerNormFunction (NAFNet_base/basicsr/models/archs/arch_util.py:264-300), NHWC, C any multiple of
 * 16 bytes (8 16-bit / 4 fp32 channels) up to 256 such chunks: writes nout = w * (x - mu) / den + b and stats[M][2] = {mu, den = sqrt(var + eps)}.
 * The closed-form backward (:277-289) recomputes yhat from x and stats, adds the residual gradient dres and writes
 * per-block partials of dw / db into slab_w / slab_b ([nbp_ln_nhwc_grid(M, C, dtype)][C] each, fold with
 * nbp_reduce_slab). */
int nbp_ln_nhwc_grid(long M, int C, int dtype);
int nbp_ln_fwd_nhwc(const void* x, const float* w, const float* b, void* nout, float* stats, long M, int C, float eps,
                    int dtype, nbp_stream_t s);
int nbp_ln_bwd_nhwc(const void* dn, const void* x, const float* stats, const float* w, const void* dres, void* dx,
                    float* slab_w, float* slab_b, long M, int C, int dtype, nbp_stream_t s);
/* NCHW variants for the standalone LayerNorm2d module. */
int nbp_ln_fwd_nchw(const float* x, const float* w, const float* b, float* y, float* yhat, float* den, int N, int C,
                    long HW, float eps, nbp_stream_t s);
int nbp_ln_bwd_nchw_workspace_floats(int N, int C, long HW);
int nbp_ln_bwd_nchw(const float* dy, const float* yhat, const float* den, const float* w, float* dx, float* dw,
                    float* db, float* ws, int N, int C, long HW, nbp_stream_t s);

/* NAFBlock spatial branch: conv2 depthwise 3x3 + bias on 2C channels (NAFNet_arch.py:32-33) -> SimpleGate
 * (:22-25) -> AdaptiveAvgPool2d(1) partial sums (:38) in pool_slab [B][chunks][C]. */
int nbp_dw_chunks(int B, int H, int W, int C, int which);
/* Rows per image of the pool_slab nbp_dw_sg_pool_fwd writes for this shape and dtype ([B][rows][C]). */
int nbp_dw_fwd_slab_rows(int B, int H, int W, int C, int dtype);
int nbp_dw_sg_pool_fwd(const void* t1, const float* wdw, const float* bdw, void* t2, void* g, float* pool_slab, int B,
                       int H, int W, int C, int dtype, nbp_stream_t s);
/* The deep levels' conv1 -> conv2 depthwise -> SimpleGate -> pool in one launch (NAFNet_arch.py:59-68, whole-image
 * tiles, 16-bit storage): t1 = n1 W1^T + b1 [B*H*W][2C] (the tape), t2 (NULL: not kept), g [B*H*W][C] and the pool
 * sums pool[B][C] (a one-row pool_slab: nbp_sca_fwd with chunks = 1).  t1 / t2 / g bitwise those of nbp_gemm_bf16 +
 * nbp_dw_sg_pool_fwd; pool up to fp32 summation order.  nbp_c1dw_supported(H, W, C, dtype) is 1 for the shape served
 * (16 x 16 at C 512). */
int nbp_c1dw_supported(int H, int W, int C, int dtype);
int nbp_c1_dw_sg_pool(const void* n1, const void* w1, const float* b1, const float* wdw, const float* bdw, void* t1,
                      void* t2, void* g, float* pool, int B, int H, int W, int C, int dtype, nbp_stream_t s);
/* Levels 0 / 1 (C 32 / 64, 16-bit) with the 2C-wide tape kept on chip (NAFNet_arch.py:59-68: conv1 -> conv2 (dw 3x3)
 * -> SimpleGate -> the SCA's pool).  nbp_c1dw_fwd_tile: g = SG(dw3x3(conv1(n1))) and per-tile pool partials
 * pool_slab[B][nbp_c1dw_tile_rows(H, W, C)][C] (the `chunks` of nbp_sca_fwd); t1 / t2 are written only when given
 * (NULL: the backward rebuilds them).  w1: the 16-bit conv1 weight [2C][C].  t1, t2, g bitwise equal the skinny conv1
 * + nbp_dw_sg_pool_fwd; pool equal up to fp32 summation order.
 * nbp_c1dw_bwd_tile: replaces nbp_sca_sg_dw_bwd given n1 instead of t1 / t2 (rebuilt on chip, bitwise the forward's):
 * dt1 = dw3x3^T(dt2), dt2 = (dg t2[C:], dg t2[:C]), dg = dh a + ds / HW; dwdw / dbdw as nbp_sca_sg_dw_bwd (per-tile
 * slabs in ws, nbp_c1dw_bwd_workspace_floats, reduced with nbp_reduce_slab: deferred when deferral is on).  dt1 bitwise
 * equal to nbp_sca_sg_dw_bwd on the stored tape; dwdw / dbdw up to fp32 summation order.
 * nbp_c1dw_tile_supported(B, H, W, C, dtype) is 1 for the shapes served (16-bit, C 32 / 64, and B*H*W*C*4 bytes within the
 * kernels' 32-bit buffer offsets; larger levels take the stored-tape kernels). */
int nbp_c1dw_tile_supported(int B, int H, int W, int C, int dtype);
int nbp_c1dw_tile_rows(int H, int W, int C);
int nbp_c1dw_fwd_tile(const void* n1, const void* w1, const float* b1, const float* wdw, const float* bdw, void* t1,
                      void* t2, void* g, float* pool_slab, int B, int H, int W, int C, int dtype, nbp_stream_t s);
size_t nbp_c1dw_bwd_workspace_floats(int B, int H, int W, int C);
int nbp_c1dw_bwd_tile(const void* dh, const float* a, const float* ds, const void* n1, const void* w1, const float* b1,
                      const float* wdw, const float* bdw, void* dt1, float* dwdw, float* dbdw, float* ws, int B, int H,
                      int W, int C, int dtype, nbp_stream_t s);
/* nbp_c1dw_bwd_tile with the SCA backward (nbp_sca_bwd_fused) folded in, as nbp_sca_dw_bwd does for the stored-tape
 * levels: ds of each workgroup's 32 gate channels from the channel-dot partials (da_slab [B][chunks][C]) first, rows of
 * dwsca / dbsca spread over the workgroups.  B <= 256; the default tile variant (NBP_C1DW_BWD_TH / _BAL unset). */
int nbp_sca_c1dw_bwd_tile(const void* dh, const float* a, const float* da_slab, int chunks, const float* wsca,
                          const float* mean, float* dwsca, float* dbsca, const void* n1, const void* w1, const float* b1,
                          const float* wdw, const float* bdw, void* dt1, float* dwdw, float* dbdw, float* ws, int B,
                          int H, int W, int C, int dtype, nbp_stream_t s);
/* SCA 1x1 conv on the pooled vector (:39-41): mean[B][C], a[B][C] = W mean + b. */
int nbp_sca_fwd(const float* pool_slab, int chunks, const float* wsca, const float* bsca, float* mean, float* a, int B,
                int HW, int C, nbp_stream_t s);
/* per-image channel sums slab[b][chunk][c] = sum_p x*y (y may be NULL). */
int nbp_img_chan_dot(const void* x, const void* y, float* slab, int B, int H, int W, int C, int dtype, nbp_stream_t s);
/* SCA backward: da[B][C] = the reduced img_chan_dot slab, ds = da . W (the pooled-vector gradient).  The weight
   gradients dW = da^T mean, db = sum_b da are a K = B weight-gradient GEMM (nbp_wgrad_f32 on da and mean). */
int nbp_sca_bwd(const float* da_slab, int chunks, const float* wsca, float* da, float* ds, int B, int C,
                nbp_stream_t s);
/* The whole SCA backward in one launch: ds = da . W with da reduced from the img_chan_dot slab, and the SCA weight
   gradients dW[o][i] = sum_b da[b][o] mean[b][i], db[o] = sum_b da[b][o] written in place (replaces nbp_sca_bwd +
   the K = B nbp_wgrad_f32; NAFNet_arch.py:39-41,67). */
int nbp_sca_bwd_fused(const float* da_slab, int chunks, const float* wsca, const float* mean, float* ds, float* dW,
                      float* db, int B, int C, nbp_stream_t s);
/* 1 when the LDS-tiled depthwise kernels serve C channels at this dtype (then nbp_dw_sg_pool_fwd may be given
   t2 = NULL when no backward follows). */
int nbp_dw_tiled(int C, int dtype);
/* dg = dh*a + ds/HW, then SimpleGate backward into dt2 [M][2C]. */
int nbp_sca_sg_bwd(const void* dh, const float* a, const float* ds, const void* t2, void* dt2, long M, int C, int HW,
                   int dtype, nbp_stream_t s);
/* depthwise 3x3 backward: dt1, dW [2C][9], db [2C]. */
size_t nbp_dw_bwd_workspace_floats(int B, int H, int W, int C);
int nbp_dw_bwd(const void* dt2, const void* t1, const float* wdw, void* dt1, float* dwdw, float* dbdw, float* ws,
               int B, int H, int W, int C, int dtype, nbp_stream_t s);
/* SCA + SimpleGate backward fused into the depthwise backward (NAFNet_arch.py:64-67 adjoint): dt2 is formed in LDS as
   (dg * t2[:, C:], dg * t2[:, :C]) with dg = dh * a[b] + ds[b] / (H*W), never written to HBM; outputs as nbp_dw_bwd.
   Requires C % 16 == 0 (bf16) or C % 8 == 0 (fp32); ws as nbp_dw_bwd_workspace_floats. */
int nbp_sca_sg_dw_bwd(const void* dh, const float* a, const float* ds, const void* t2, const void* t1, const float* wdw,
                      void* dt1, float* dwdw, float* dbdw, float* ws, int B, int H, int W, int C, int dtype,
                      nbp_stream_t s);
/* The SCA backward (nbp_sca_bwd_fused) folded into nbp_sca_sg_dw_bwd: each workgroup reduces its image's channel-dot
 * partials (da_slab [B][chunks][C]) and forms ds of its own gate channels (ds[b][i] = sum_o W_sca[o][i] da[b][o]) before
 * the fused depthwise backward; rows o of dwsca / dbsca (= sum_b da[b][o] mean[b][:] / da[b][o]) are spread over the
 * workgroups.  16-bit, C a multiple of 16, C <= 1024, B <= 256.  Replaces, for the levels with the stored tape, the
 * reference's SCA backward (NAFNet_arch.py:39-41, 67) and the two launches; ds / dW / db equal theirs up to fp32
 * summation order. */
int nbp_sca_dw_bwd(const void* dh, const float* a, const float* da_slab, int chunks, const float* wsca, const float* mean,
                   float* dwsca, float* dbsca, const void* t2, const void* t1, const float* wdw, void* dt1, float* dwdw,
                   float* dbdw, float* ws, int B, int H, int W, int C, int dtype, nbp_stream_t s);

/* SimpleGate on the FFN half (NAFNet_arch.py:75): g = t[:C]*t[C:], and its backward. */
/* layout 0: t = [t_a | t_b] halves; layout 1: pairs (a_c, b_c) interleaved (the internal conv4 channel order). */
int nbp_sg_fwd(const void* t, void* g, long M, int C, int layout, int dtype, nbp_stream_t s);
int nbp_sg_bwd(const void* dg, const void* t, void* dt, long M, int C, int layout, int dtype, nbp_stream_t s);
/* layer-scale residual gradients (NAFNet_arch.py:72,80): ds = d*scale, slab partials of sum d*t (dbeta/dgamma). */
int nbp_scale_dot_grid(long M, int C);
int nbp_scale_dot(const void* d, const void* t, const float* scale, void* ds, float* slab, long M, int C, int dtype,
                  nbp_stream_t s);
int nbp_nchw_to_nhwc(const float* x, float* y, int N, int C, long HW, nbp_stream_t s);
int nbp_nhwc_to_nchw(const float* x, float* y, int N, int C, long HW, nbp_stream_t s);
int nbp_add(const void* a, const void* b, void* y, long n, int dtype, nbp_stream_t s);

/* intro conv 3x3 (NAFNet_arch.py:88-89,136) on the check_image_size zero-padded grid (:157-162): NCHW image ->
 * NHWC features [B][Hp][Wp][Cf]; backward gives dW, db and (optional) d image. */
int nbp_intro_fwd(const float* img, const float* w, const float* bias, void* out, int B, int Cimg, int H0, int W0,
                  int Hp, int Wp, int Cf, int dtype, nbp_stream_t s);
size_t nbp_intro_bwd_workspace_floats(int B, int Cimg, int Hp, int Wp, int Cf);
int nbp_intro_bwd(const float* img, const void* dout, const float* w, float* dw, float* db, float* dimg, float* ws,
                  int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s);
/* ending conv 3x3 + global residual + crop (NAFNet_arch.py:90-91,152-155): NHWC features -> NCHW image. */
int nbp_ending_fwd(const void* feat, const float* w, const float* bias, const float* img, float* out, int B, int Cimg,
                   int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s);
size_t nbp_ending_bwd_workspace_floats(int B, int Cimg, int H0, int W0, int Cf);
int nbp_ending_bwd(const float* dy, const void* feat, const float* w, void* dfeat, float* dw, float* db, float* ws,
                   int B, int Cimg, int H0, int W0, int Hp, int Wp, int Cf, int dtype, nbp_stream_t s);

/* ------------------------------------------------------------------ HybridLoss terms (NCHW) */
/* mode 0: nn.L1Loss (NewBP_model/losses.py:249,332); mode 1: Charbonnier sqrt(d^2+eps)
 * (NAFNet_base/basicsr/models/losses/losses.py:29-31).  clamp_a/clamp_b apply clamp(0,1) to the inputs. */
size_t nbp_pix_workspace_doubles(long n);
int nbp_pix_loss_fwd(const float* a, const float* b, long n, int mode, float eps, int clamp_a, int clamp_b, double* ws,
                     float* loss, nbp_stream_t s);
int nbp_pix_loss_bwd(const float* a, const float* b, long n, int mode, float eps, int clamp_a, int clamp_b,
                     const float* up, float* ga, nbp_stream_t s);
/* SSIMLoss (losses.py:146-155 -> kornia 0.6.12 ssim_loss, window 11, sigma 1.5, reflect pad): the loss map
 * clamp((1 - ssim) / 2, 0, 1) reduced by `reduction` 0 = 'mean' (loss[0]), 1 = 'sum' (loss[0]) or 2 = 'none' (lmap
 * [N][C][H][W]; loss may be null).  want_grad keeps the gradient coefficients in ws for nbp_ssim_loss_bwd, which writes
 * gx = d/dx: scaled by up[0] (mean / sum) or, with up_map (reduction 'none'), by the per-pixel upstream map.  The map
 * is symmetric in (x, y): d/dy is the same pair of calls with x and y swapped.  With want_grad = 1, loss and lmap may
 * both be null: the call then only fills ws (the d/dy coefficients of that swapped call, no reduction, no map). */
size_t nbp_ssim_workspace_floats(long n);
int nbp_ssim_loss_fwd(const float* x, const float* y, int N, int C, int H, int W, int window, float max_val,
                      int clamp_in, int want_grad, int reduction, float* ws, float* loss, float* lmap, nbp_stream_t s);
int nbp_ssim_loss_bwd(const float* x, const float* y, int N, int C, int H, int W, int clamp_in, const float* up,
                      const float* up_map, float* ws, float* gx, nbp_stream_t s);

/* ------------------------------------------------------------------ colour difference (NCHW sRGB [B][3][H][W] fp32) */
/* DeltaE00Loss (NewBP_model/losses.py:92-143): out[0] = mean over pixels of the loss-form CIEDE2000 between
   rgb_to_lab(clamp01 gen) and rgb_to_lab(clamp01 tgt) (kornia 0.6.12 conversion; clamp = 0 skips the clamps);
   ws: nbp_de00_workspace_doubles(B*H*W) doubles.  The backward writes dgen = up[0] / (B*H*W) * d dE / d gen; the
   loss is symmetric in (gen, tgt), so d / d tgt is the backward with the two swapped. */
size_t nbp_de00_workspace_doubles(long npix);
int nbp_de00_loss_fwd(const float* gen, const float* tgt, int B, int H, int W, int clamp, float eps, double* ws,
                      float* out, nbp_stream_t s);
int nbp_de00_loss_bwd(const float* gen, const float* tgt, int B, int H, int W, int clamp, float eps, const float* up,
                      float* dgen, nbp_stream_t s);
/* deltaE2000_map (metrics/color_error.py:235-267 -> _deltaE00_lab_map :105-210): map [B][H][W]. */
int nbp_de00_metric_map(const float* pred, const float* tgt, int B, int H, int W, float kL, float kC, float kH,
                        float eps, float* map, nbp_stream_t s);
/* Per-pixel CIEDE2000 on Lab inputs [B][3][H][W] -> out [B][H][W]: form 0 = the loss form (losses.py:98-136,
   eps), 1 = the metric form (color_error.py:105-210, kL kC kH eps). */
int nbp_de00_lab(const float* lab1, const float* lab2, int B, int H, int W, int form, float kL, float kC, float kH,
                 float eps, float* out, nbp_stream_t s);
/* Gradient of the loss form on Lab inputs (DeltaE00Loss._ciede2000's autograd): d1 = g [B][H][W] * d dE / d lab1
   (forward-mode AD per pixel).  The form is symmetric: d / d lab2 = the same call with lab1 and lab2 swapped. */
int nbp_de00_lab_bwd(const float* lab1, const float* lab2, int B, int H, int W, float eps, const float* g, float* d1,
                     nbp_stream_t s);
/* kornia rgb_to_lab of NCHW sRGB into lab [B][3][H][W]. */
int nbp_rgb_to_lab(const float* rgb, int B, int H, int W, float* lab, nbp_stream_t s);

/* ------------------------------------------------------------------ validation metrics (rows 26-27) */
/* Per-sample PSNR over N samples of L fp32 elements: psnr_linear (metrics/linear.py:140-215, diff_double = 0: fp32
   difference squared in float64) or calculate_psnr (metrics/psnr.py:18-67, diff_double = 1, N = 1); mse / psnr are
   float64 [N] (mse may be null); inf where mse <= eps.  ws: nbp_psnr_workspace_doubles(N, L) doubles. */
size_t nbp_psnr_workspace_doubles(int N, long L);
int nbp_psnr(const float* pred, const float* tgt, int N, long L, double data_range, double eps, int diff_double,
             double* ws, double* mse, double* psnr, nbp_stream_t s);
/* calculate_ssim input alignment (metrics/ssim.py): BT.601 luma of NCHW RGB (color_space='y', :119-131) -> [N,1,H,W],
 * and F.interpolate(bilinear / bicubic, align_corners=False) of `planes` Hi x Wi planes to Ho x Wo (resize_policy
 * 'resize', :144-152; torch's CPU source-index and weight formulas). */
int nbp_luma_bt601(const float* x, int N, int H, int W, float* y, nbp_stream_t s);
int nbp_resize_planes(const float* x, long planes, int Hi, int Wi, int Ho, int Wo, int cubic, float* y, nbp_stream_t s);
/* Windowed SSIM per-plane means out [N*C] float64: ssim_linear (metrics/linear.py:218-324: clamp_var = 1, crop = 0,
   eps) or the torchmetrics-1.2.0 form behind calculate_ssim (metrics/ssim.py:341-377: clamp_var = 0, eps = 0,
   crop = 1: the k/2 border of the map is excluded).  win: the k normalised 1-D window weights (device);
   pad_mode 0 reflect, 1 replicate, 2 circular, 3 constant(0). */
size_t nbp_ssim_linear_workspace_floats(int N, int C, int H, int W);
int nbp_ssim_linear(const float* pred, const float* tgt, int N, int C, int H, int W, const float* win, int k,
                    int pad_mode, float c1, float c2, float eps, int clamp_var, int crop, float* ws, double* out,
                    nbp_stream_t s);
/* |Sobel| of channel 0 of lab [B][3][H][W] (zero padding, +1e-12 under the root; color_error.py:296-302). */
int nbp_sobel_mag(const float* lab, int B, int H, int W, float* out, nbp_stream_t s);

/* ------------------------------------------------------------------ VGG feature losses (rows 19, 22) */
/* 3x3 zero-padded conv over NHWC bf16 as an implicit GEMM on bf16 MFMA (K = 9*Cin gathered on the fly):
   y = epi(sum_{t,c} x[i + t/3 - 1][j + t%3 - 1][c] * w[n][t][c]); mode 0 = + bias then ReLU, 1 = + bias,
   2 = keep where R > 0 (ReLU mask of a saved post-ReLU map; the input-gradient pass uses the tap-flipped,
   transposed weights).  Cin, Cout multiples of 8; y bf16 (y_dtype 1) or fp32 (y_dtype 0, mode 1). */
int nbp_conv3x3_bf16(const void* x, int B, int H, int W, int Cin, const void* w, int Cout, const float* bias, int mode,
                     const void* R, void* y, int y_dtype, int dtype, nbp_stream_t s);
/* General zero-padded KH x KW / stride conv over NHWC maps (LPIPS(net='alex') trunk, lpips 0.1.4 /
   torchvision alexnet.features: 11x11/4 pad 2, 5x5 pad 2, 3x3 pad 1), implicit GEMM on the MFMA kernels:
   y [B][Ho][Wo][Cout] = epi(sum_{ki,kj,c} x[b][oi*stride + ki - pad][oj*stride + kj - pad][c] w[n][ki*KW+kj][c]),
   Ho = (H + 2 pad - KH) / stride + 1; epi as nbp_conv3x3_bf16: mode 0 bias + ReLU, 1 bias (or none), 2 ReLU-mask by
   R (y = acc where R > 0: the stride-1 input gradient with tap-flipped [Cin][tap][Cout] weights).  Cin, Cout multiples
   of 8; dtype 0 fp32 / 1 bf16 / 2 fp16 (x, w, R, y). */
int nbp_conv2d_16(const void* x, int B, int H, int W, int Cin, const void* w, int Cout, int KH, int KW, int stride,
                  int pad, const float* bias, int mode, const void* R, void* y, int dtype, nbp_stream_t s);
/* k x k / stride max pool without padding (torchvision AlexNet's MaxPool2d(3, 2)), NHWC; idx (optional) = the window
   position (row-major, first maximum as torch's max_pool2d) of each output for the backward. */
int nbp_maxpool_k_fwd(const void* x, int B, int H, int W, int C, int k, int stride, void* y, unsigned char* idx,
                      int dtype, nbp_stream_t s);
/* dx [B][H][W][C] = (sum of dy over the windows whose argmax is this input) * (post_in > 0): the pool input is a
   post-ReLU map, its ReLU mask rides along (as nbp_maxpool2_bwd). */
int nbp_maxpool_k_bwd(const void* dy, const unsigned char* idx, const void* post_in, int B, int H, int W, int C, int k,
                      int stride, void* dx, int dtype, nbp_stream_t s);
/* Input gradient of LPIPS alex's first conv (11x11, stride 4, pad 2, Cin padded 3 -> 8), a direct transposed conv:
   d8 [B][H][W][8] fp32 (channels 0..2; 3..7 zero) = sum over the output taps that read (i, j) of
   dpre[b][oi][oj][n] * w[n][ki*11+kj][c].  dpre [B][Ho][Wo][Cout] in `dtype`; w fp32 [Cout][121][8]. */
int nbp_alex_conv0_input_grad(const void* dpre, const float* w, int B, int H, int W, int Ho, int Wo, int Cout,
                              float* d8, int dtype, nbp_stream_t s);
/* PerceptualLoss input (losses.py:56-66): NCHW fp32 sRGB -> NHWC bf16 [B][H][W][8] = (clamp01(x) - m) / s, c >= 3
   zero.  The input gradient maps d[B][H][W][8] fp32 back to NCHW (/ s, clamp mask). */
int nbp_vgg_prep(const float* x, int B, int H, int W, int clamp, float m0, float m1, float m2, float s0, float s1,
                 float s2, void* y, int dtype, nbp_stream_t s);
int nbp_vgg_input_grad(const float* d8, const float* x, int B, int H, int W, int clamp, float s0, float s1, float s2,
                       float* dx, nbp_stream_t s);
/* 2x2 max pool over NHWC bf16 (floor) with the argmax (window order, first maximum); the backward scatters dy to
   the argmax and applies the ReLU mask of the (post-ReLU) pool input. */
int nbp_maxpool2_fwd(const void* x, int B, int H, int W, int C, void* y, unsigned char* idx, int dtype, nbp_stream_t s);
int nbp_maxpool2_bwd(const void* dy, const unsigned char* idx, const void* post_in, int B, int H, int W, int C, void* dx,
                     int dtype, nbp_stream_t s);
/* LPIPS tap (lpips 0.1.4 net='vgg'): out[n] (+)= mean over the HW pixels of sum_c w_c (u_c - v_c)^2 with
   u = a / (|a|_C + 1e-10), v likewise for b (a, b: NHWC bf16 [N][HW][C]); the backward writes
   da = up[n] * d out[n] / da (zero for all-zero pixels).  ws: nbp_lpips_tap_workspace_doubles(N, HW). */
size_t nbp_lpips_tap_workspace_doubles(int N, long HW);
int nbp_lpips_tap_fwd(const void* a, const void* b, const float* w, int N, long HW, int C, int accumulate, double* ws,
                      float* out, int dtype, nbp_stream_t s);
int nbp_lpips_tap_bwd(const void* a, const void* b, const float* w, int N, long HW, int C, const float* up, void* da,
                      int dtype, nbp_stream_t s);
/* d += g * (post > 0) over n bf16 elements (a tapped post-ReLU map's gradient joining the backward walk). */
int nbp_add_relu_masked(void* d, const void* g, const void* post, long n, int dtype, nbp_stream_t s);
/* Feature distance over n bf16 elements: out = scale * sum (a-b)^2 (mode 0) or |a-b| (mode 1); the backward writes
   da = up[0] * scale * d/da, optionally masked by (a > 0) (the last ReLU).  ws: nbp_feat_dist_workspace_doubles(n). */
size_t nbp_feat_dist_workspace_doubles(long n);
int nbp_feat_dist_fwd(const void* a, const void* b, long n, int mode, double scale, double* ws, float* out,
                      int dtype, nbp_stream_t s);
int nbp_feat_dist_bwd(const void* a, const void* b, long n, int mode, float scale, int relu_mask, const float* up,
                      void* da, int dtype, nbp_stream_t s);

/* ------------------------------------------------------------------ optimizer (image_restoration_model.py:313-320) */
/* Everything between backward and the AdamW update, decided on the device (no host sync, graph-replayable):
   GradScaler.unscale_ + clip_grad_norm_(params, max_norm) + the inf/nan verdict + the AdamW step count / bias
   corrections + GradScaler.update (torch.amp semantics: backoff on a non-finite step, growth every
   growth_interval finite steps).  grad = sum over ranks of the (loss-scaled) gradients; grad_scale = 1/world.
     state[8]: 0 ||averaged unscaled grad||, 1 gradient multiplier (clip coef * grad_scale / S), 2 skip flag (1 =
               non-finite gradient: the AdamW update is skipped), 3 lr / (1 - beta1^t), 4 sqrt(1 - beta2^t), 5 lr,
               6 the loss scale S of this step
     ctl[4] (int): 0 AdamW steps taken t, 1 growth tracker, 2 skipped steps
     lr: device float (this iteration's scheduled lr; written by the host between graph replays)
     scaler[4] (NULL = no loss scaling): {S, growth_factor, backoff_factor, growth_interval}, updated in place
     up[n_up] = up_base[n_up] * S_new: the loss terms' upstream gradients for the next step (n_up may be 0).
   ws: nbp_clip_workspace_doubles(n). */
size_t nbp_clip_workspace_doubles(long n);
int nbp_optim_prepare(const float* grad, long n, float grad_scale, float max_norm, double* ws, const float* lr,
                      float beta1, float beta2, float* state, int* ctl, float* scaler, float* up, const float* up_base,
                      int n_up, nbp_stream_t s);
/* torch.optim.AdamW step (decoupled weight decay) over the flat buffer with gradient * state[1], lr = state[5] and
   the bias corrections state[3..4]; a no-op when state[2] != 0 (scaler.step's skip). */
int nbp_adamw_apply(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n, const float* state,
                    float beta1, float beta2, float eps, float weight_decay, nbp_stream_t s);

/* ------------------------------------------------------------------ SID input path
 * Host-side (no GPU, no stream): the reference reads PNG bytes from LMDB (basicsr FileClient 'lmdb',
 * NAFNet_base/basicsr/data/sony_sid_lmdb_dataset.py:110-125,150-156) or disk and decodes them with
 * cv2.imdecode(IMREAD_UNCHANGED) (:38-56).  An LMDB environment is opened read-only (mmap) and named by an int
 * handle; nbp_lmdb_get returns a pointer into the map (*vlen = -1: key absent, as txn.get -> None). */
int nbp_lmdb_open(const char* path);
int nbp_lmdb_close(int handle);
int nbp_lmdb_stat(int handle, long* entries, long* psize);
int nbp_lmdb_get(int handle, const char* key, int klen, const void** val, long* vlen);
/* IHDR of a PNG: channels = those of the cv2 IMREAD_UNCHANGED array (1 gray, 3 RGB / palette, 4 with alpha or tRNS),
 * depth = 8 or 16 after palette / low-depth expansion. */
int nbp_png_info(const void* buf, long len, int* h, int* w, int* channels, int* depth);
/* 3-channel PNG -> uint16 [crop_h][crop_w][3] in the file's R, G, B order, 8-bit values * 257 (the uint8 promotion
 * of _load_png_uint16, :45-47); crop_h <= 0 decodes the whole image.  The crop is _maybe_random_crop's window
 * (:162-192). */
int nbp_png_decode_rgb16(const void* buf, long len, void* out, int top, int left, int crop_h, int crop_w);
/* n PNGs decoded and cropped on nthreads host threads into out[n][crop_h][crop_w][3]. */
int nbp_png_decode_batch(int n, const void* const* bufs, const long* lens, const int* tops, const int* lefts,
                         int crop_h, int crop_w, void* out, int nthreads);
/* Device: uint16 NHWC crops -> lq (= short = short_obs) = clip(short/65535 * ratio[b], 0, 1), short_raw =
 * short/65535, long_raw (= gt = long) = long/65535, NCHW float32 [B][3][H][W] (sony_sid_lmdb_dataset.py:207-218). */
int nbp_sid_to_float(const void* short_u16, const void* long_u16, const float* ratio, int B, int H, int W, float* lq,
                     float* short_raw, float* long_raw, nbp_stream_t s);

#ifdef __cplusplus
}
#endif

#endif /* NBP_H_ */
