// Throughput of the fp32 MFMAs on gfx950: every wave issues N MFMAs over 4 independent accumulator chains
// (hipcc --offload-arch=gfx950 -O3 scripts/mfma_f32_probe.hip -o mfma_f32_probe && ./mfma_f32_probe)
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int KIND, int CH>
__global__ __launch_bounds__(256) void probe(float* out, int n, float a0) {
  floatx16 acc[CH];
  floatx4 acc4[CH];
  for (int j = 0; j < CH; ++j) { for (int r = 0; r < 16; ++r) acc[j][r] = 0.f; for (int r = 0; r < 4; ++r) acc4[j][r] = 0.f; }
  float a = a0 + threadIdx.x, b = a0 * 0.5f + blockIdx.x;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (KIND == 0) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
      else acc4[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc4[j], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int j = 0; j < CH; ++j) { for (int r = 0; r < 16; ++r) s += acc[j][r]; for (int r = 0; r < 4; ++r) s += acc4[j][r]; }
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int KIND, int CH>
void run(float* out, int blocks, int n) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  probe<KIND, CH><<<blocks, 256>>>(out, n, 1.f);
  hipEventRecord(e0);
  probe<KIND, CH><<<blocks, 256>>>(out, n, 1.f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double mfma = (double)blocks * 4 * n * CH;
  const double flop = mfma * (KIND == 0 ? 32.0 * 32 * 2 * 2 : 16.0 * 16 * 4 * 2);
  printf("%s chains %d blocks %d: %.1f us, %.1f cycles per MFMA per SIMD (2.4 GHz, 1024 SIMDs), %.1f TFLOP/s\n",
         KIND == 0 ? "32x32x2f32" : "16x16x4f32", CH, blocks, ms * 1e3, ms * 1e-3 * 2.4e9 * 1024 / mfma, flop / (ms * 1e-3) / 1e12);
}
int main() {
  float* out;
  hipMalloc(&out, 8192 * 256 * 4);
  run<0, 1>(out, 1024, 512); run<0, 4>(out, 1024, 128); run<0, 4>(out, 2048, 128);
  run<1, 1>(out, 1024, 512); run<1, 4>(out, 1024, 128); run<1, 4>(out, 2048, 128);
  hipFree(out);
  return 0;
}
