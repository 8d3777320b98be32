// Cost of a dependent phase boundary on MI355X: P dependent launches of a small kernel (captured in one HIP graph)
// vs ONE persistent launch running the same P phases separated by a grid barrier (device-scope release / acquire,
// bounded spin).  Each phase: every workgroup mixes its own slice with its neighbour's slice of the previous phase's
// buffer (a true cross-workgroup dependency), W floats per workgroup.
//   hipcc -O3 --offload-arch=gfx950 scripts/phase_probe.hip -o build/phase_probe && build/phase_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

__device__ __forceinline__ void phase_body(const float* in, float* out, int W, int wg, int nwg, int nb) {
  const float* a = in + (long)wg * W;
  const float* b = in + (long)((wg + nb) % nwg) * W;  // the workgroup nb ids away (nb = 8: the same XCD)
  float* o = out + (long)wg * W;
  for (int i = threadIdx.x * 4; i < W; i += blockDim.x * 4) {
    const float4 x = *reinterpret_cast<const float4*>(a + i), y = *reinterpret_cast<const float4*>(b + i);
    *reinterpret_cast<float4*>(o + i) = make_float4(0.5f * (x.x + y.x), 0.5f * (x.y + y.y), 0.5f * (x.z + y.z),
                                                    0.5f * (x.w + y.w));
  }
}

__global__ void step_kernel(const float* in, float* out, int W, int nb) {
  phase_body(in, out, W, blockIdx.x, gridDim.x, nb);
}

// grid barrier: one arrival counter + generation word, thread 0 of each workgroup; device-scope fences publish the
// phase's stores (the workgroups sit on 8 XCDs with separate L2s).  The spin is bounded: on timeout the flag is set
// and the kernel finishes (wrong data, no hang).
__device__ __forceinline__ void grid_barrier(unsigned* count, unsigned* gen, unsigned n, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned g = __hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == n - 1) {
      __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(gen, g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long spins = 0;
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1L << 24)) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

__global__ void persistent_kernel(float* b0, float* b1, int W, int P, unsigned* count, unsigned* gen, int* err, int nb) {
  for (int p = 0; p < P; ++p) {
    const float* in = (p & 1) ? b1 : b0;
    float* out = (p & 1) ? b0 : b1;
    phase_body(in, out, W, blockIdx.x, gridDim.x, nb);
    grid_barrier(count, gen, gridDim.x, err);
  }
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int nwg = ncu;  // one workgroup per CU (tiny LDS / registers: all co-resident)
  const int P = 200;
  float *b0, *b1;
  unsigned *count, *gen;
  int* err;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("CUs %d, workgroups %d x 256 threads, %d phases\n", ncu, nwg, P);
  for (int W : {1024, 16384}) {  // 4 KB or 64 KB per workgroup per phase
    const size_t bytes = (size_t)nwg * W * sizeof(float);
    CK(hipMalloc(&b0, bytes));
    CK(hipMalloc(&b1, bytes));
    CK(hipMemset(b0, 0, bytes));
    CK(hipMemset(b1, 0, bytes));
    CK(hipMalloc(&count, 4));
    CK(hipMalloc(&gen, 4));
    CK(hipMalloc(&err, 4));
    for (int nb : {1, 8}) {
      // P dependent launches captured in one graph
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
      for (int p = 0; p < P; ++p)
        step_kernel<<<nwg, 256, 0, st>>>((p & 1) ? b1 : b0, (p & 1) ? b0 : b1, W, nb);
      CK(hipStreamEndCapture(st, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, st));
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(e0, st));
      CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms_g = 0.f;
      CK(hipEventElapsedTime(&ms_g, e0, e1));
      // one persistent launch
      float ms_p = 0.f;
      int herr = 0;
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemsetAsync(count, 0, 4, st));
        CK(hipMemsetAsync(gen, 0, 4, st));
        CK(hipMemsetAsync(err, 0, 4, st));
        CK(hipEventRecord(e0, st));
        persistent_kernel<<<nwg, 256, 0, st>>>(b0, b1, W, P, count, gen, err, nb);
        CK(hipEventRecord(e1, st));
        CK(hipStreamSynchronize(st));
        CK(hipEventElapsedTime(&ms_p, e0, e1));
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      }
      printf("W %5d floats/wg, neighbour +%d: %d launches in a graph %.2f us/phase | persistent + grid barrier %.2f us/phase%s\n",
             W, nb, P, ms_g * 1e3f / P, ms_p * 1e3f / P, herr ? " (BARRIER TIMEOUT)" : "");
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
    CK(hipFree(b0));
    CK(hipFree(b1));
    CK(hipFree(count));
    CK(hipFree(gen));
    CK(hipFree(err));
  }
  return 0;
}
