// Implicit-GEMM convolutions of the VGG / LPIPS trunks: 16-bit on the DMA GEMM kernel of gemm16_impl.h, fp32 (the
// parity mode, dtype 0) on the fp32 MFMA GEMM of gemm.hip (nbp::conv_f32).
#include "gemm16_impl.h"

extern "C" {

// 3x3 zero-padded convolution over NHWC 16-bit maps as an implicit GEMM on the 16-bit MFMA kernel:
//   y[b][i][j][n] = epi( sum_{t, c} x[b][i + t/3 - 1][j + t%3 - 1][c] * w[n][t][c] (+ bias[n]) )
// epi: mode 0 bias + ReLU, 1 bias only, 2 ReLU-mask by R (y = acc where R > 0 else 0; no bias).  x, w, R and a
// 16-bit y share the type `dtype` (1 bf16, 2 fp16); y is that type (y_dtype 1) or fp32 (y_dtype 0, mode 1 only).
// dtype 0: x, w, R, y all fp32 (y_dtype 0).
// Cin % 8 == 0 (pad the channel dimension), Cout % 8 == 0.
int nbp_conv3x3_bf16(const void* x, int B, int H, int W, int Cin, const void* w, int Cout, const float* bias, int mode,
                     const void* R, void* y, int y_dtype, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && w && y && B > 0 && H > 0 && W > 0, "nbp_conv3x3_bf16: bad args");
  NBP_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "nbp_conv3x3_bf16: Cin and Cout must be multiples of 8 (%d, %d)", Cin,
              Cout);
  NBP_REQUIRE(dtype >= 0 && dtype <= 2, "nbp_conv3x3_bf16: dtype 0 (fp32), 1 (bf16) or 2 (fp16)");
  NBP_REQUIRE(mode >= 0 && mode <= 2 && (mode != 2 || R) && (dtype == 0 ? y_dtype == 0 : (y_dtype == 1 || mode == 1)),
              "nbp_conv3x3_bf16: mode / R / y_dtype");
  if (dtype == 0)
    return conv_f32(static_cast<const float*>(x), B, H, W, Cin, static_cast<const float*>(w), Cout, 3, 3, 1, 1, bias,
                    mode, static_cast<const float*>(R), static_cast<float*>(y), S(s));
  const long M = (long)B * H * W;
  NBP_REQUIRE(M < (1L << 31), "nbp_conv3x3_bf16: too many pixels");
  GemmPB p{x, 0, nullptr, 1, w, 9L * Cin, y, Cout, (int)M, Cout, 9 * Cin, H, W, Cin,
           mode == 2 ? nullptr : bias, mode == 2 ? R : nullptr, nullptr, nullptr};
  p.tap_tile = Cin % 64 == 0;  // a K-tile inside one tap: the tap is per stage, not a per-lane division
  p.tile_map = 1;  // XCD-contiguous M runs: +5-10 % on the 128 x 128 / 128 x 64 VGG tiles
  hipStream_t st = S(s);
  if (dtype == 2) {
    using T16 = _Float16;
    if (mode == 0) dispatch<AM_IM2COL, CM_RELU, T16, T16, T16>(p, st);
    else if (mode == 2) dispatch<AM_IM2COL, CM_MASK, T16, T16, T16>(p, st);
    else if (y_dtype == 1) dispatch<AM_IM2COL, CM_PLAIN, T16, T16, T16>(p, st);
    else dispatch<AM_IM2COL, CM_PLAIN, T16, float, T16>(p, st);
  } else {
    using T16 = __bf16;
    if (mode == 0) dispatch<AM_IM2COL, CM_RELU, T16, T16, T16>(p, st);
    else if (mode == 2) dispatch<AM_IM2COL, CM_MASK, T16, T16, T16>(p, st);
    else if (y_dtype == 1) dispatch<AM_IM2COL, CM_PLAIN, T16, T16, T16>(p, st);
    else dispatch<AM_IM2COL, CM_PLAIN, T16, float, T16>(p, st);
  }
  return check_launch("conv3x3_bf16");
}

int nbp_conv2d_16(const void* x, int B, int H, int W, int Cin, const void* w, int Cout, int KH, int KW, int stride,
                  int pad, const float* bias, int mode, const void* R, void* y, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(x && w && y && B > 0 && H > 0 && W > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0,
              "nbp_conv2d_16: bad args");
  NBP_REQUIRE(Cin % 8 == 0 && Cout % 8 == 0, "nbp_conv2d_16: Cin and Cout must be multiples of 8 (%d, %d)", Cin, Cout);
  NBP_REQUIRE(dtype >= 0 && dtype <= 2, "nbp_conv2d_16: dtype 0 (fp32), 1 (bf16) or 2 (fp16)");
  NBP_REQUIRE(mode >= 0 && mode <= 2 && (mode != 2 || R), "nbp_conv2d_16: mode / R");
  if (dtype == 0)
    return conv_f32(static_cast<const float*>(x), B, H, W, Cin, static_cast<const float*>(w), Cout, KH, KW, stride, pad,
                    bias, mode, static_cast<const float*>(R), static_cast<float*>(y), S(s));
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  NBP_REQUIRE(Ho > 0 && Wo > 0, "nbp_conv2d_16: empty output");
  const long M = (long)B * Ho * Wo;
  NBP_REQUIRE(M < (1L << 31), "nbp_conv2d_16: too many pixels");
  GemmPB p{x, 0, nullptr, 1, w, (long)KH * KW * Cin, y, Cout, (int)M, Cout, KH * KW * Cin, Ho, Wo, Cin,
           mode == 2 ? nullptr : bias, mode == 2 ? R : nullptr, nullptr, nullptr};
  p.kh = KH;
  p.kw = KW;
  p.stride = stride;
  p.pad = pad;
  p.ih = H;
  p.iw = W;
  hipStream_t st = S(s);
  if (dtype == 2) {
    using T16 = _Float16;
    if (mode == 0) dispatch<AM_CONV, CM_RELU, T16, T16, T16>(p, st);
    else if (mode == 2) dispatch<AM_CONV, CM_MASK, T16, T16, T16>(p, st);
    else dispatch<AM_CONV, CM_PLAIN, T16, T16, T16>(p, st);
  } else {
    using T16 = __bf16;
    if (mode == 0) dispatch<AM_CONV, CM_RELU, T16, T16, T16>(p, st);
    else if (mode == 2) dispatch<AM_CONV, CM_MASK, T16, T16, T16>(p, st);
    else dispatch<AM_CONV, CM_PLAIN, T16, T16, T16>(p, st);
  }
  return check_launch("conv2d_16");
}

}  // extern "C"
