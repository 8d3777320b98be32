// SID input path, device side: the decoded uint16 crops -> the reference's float32 batch.
//
// Reference: NAFNet_base/basicsr/data/sony_sid_lmdb_dataset.py:207-218 (per sample, numpy float32):
//   short_raw = short_obs.astype(float32) / 65535 ; long_raw = long_gt.astype(float32) / 65535
//   lq = short_obs = clip(short_raw * expo_ratio, 0, 1) ; gt = long_raw   (crop, then img2tensor HWC -> CHW)
// The crop commutes with these elementwise ops, so the host crops while decoding (sid_io.cpp) and only the window
// crosses PCIe, as uint16 (half the bytes of the float32 tensors).  Here: NHWC uint16 in, NCHW float32 out, one
// thread per pixel (the three planes are written with unit stride along W).  Arithmetic as numpy's: an IEEE
// float32 division by 65535 (hipcc keeps fp32 division correctly rounded), one rounded multiply by the float32
// ratio, then max / min.
#include "nbp_common.h"

namespace {

__global__ __launch_bounds__(256) void sid_to_float_kernel(const uint16_t* __restrict__ s, const uint16_t* __restrict__ l,
                                                           const float* __restrict__ ratio, int H, int W,
                                                           float* __restrict__ lq, float* __restrict__ sraw,
                                                           float* __restrict__ lraw) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, b = blockIdx.z;
  if (x >= W) return;
  const long pix = ((long)b * H + y) * W + x;
  const long plane = (long)H * W, o = (long)b * 3 * plane + (long)y * W + x;
  const float r = ratio[b];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float sv = (float)s[pix * 3 + c] / 65535.0f;
    const float lv = (float)l[pix * 3 + c] / 65535.0f;
    sraw[o + c * plane] = sv;
    lraw[o + c * plane] = lv;
    lq[o + c * plane] = fminf(fmaxf(sv * r, 0.0f), 1.0f);
  }
}

}  // namespace

extern "C" {

int nbp_sid_to_float(const void* short_u16, const void* long_u16, const float* ratio, int B, int H, int W, float* lq,
                     float* short_raw, float* long_raw, nbp_stream_t s) {
  NBP_REQUIRE(short_u16 && long_u16 && ratio && lq && short_raw && long_raw && B > 0 && H > 0 && W > 0,
              "nbp_sid_to_float: bad args");
  NBP_REQUIRE(B <= 65535 && H <= 65535, "nbp_sid_to_float: B, H <= 65535");
  const dim3 grid((W + 255) / 256, H, B);
  sid_to_float_kernel<<<grid, 256, 0, (hipStream_t)s>>>((const uint16_t*)short_u16, (const uint16_t*)long_u16, ratio,
                                                          H, W, lq, short_raw, long_raw);
  return nbp::check_launch("sid_to_float");
}

}  // extern "C"
