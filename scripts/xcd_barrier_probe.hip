// What a dependent phase boundary costs on MI355X: P dependent phases as
//   (a) P launches of a small kernel captured in one HIP graph,
//   (b) ONE persistent launch with a flat grid barrier (one device-scope arrival counter: the round-2 probe's form),
//   (c) ONE persistent launch with an XCD-hierarchical barrier (MI355X_MICROARCH.md row barrier-xcd; the hand-off
//       rules of cdna_hip_programming.md Guideline 16): every workgroup arrives on its XCC's counter; the last arriver
//       of an XCC (its leader) releases the XCC's L2 once (fence release agent + asm vmcnt(0)), arrives on the top
//       counter, polls it (one lane, relaxed sc1 loads + s_sleep), then publishes the XCC's generation word; the other
//       workgroups poll only their XCC's generation word; everyone acquires (fence acquire agent) after the match.
// Counters count monotonically within the call (target = members * epoch, epoch = phase + 1, never 0) and are zeroed
// by a memset node before every launch; XCC membership comes from HW_REG_XCC_ID in a census at the kernel's start (no
// dispatch-order or placement assumption).  Every spin is bounded: a timeout sets an error word and the kernel ends.
// Each phase: every workgroup mixes its own slice with the slice of the workgroup `nb` ids away from the previous phase
// (a true cross-workgroup, mostly cross-XCD dependency).  The persistent results are checked bitwise against (a).
//   hipcc -O3 --offload-arch=gfx950 scripts/xcd_barrier_probe.hip -o build/xcd_barrier_probe && build/xcd_barrier_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef __attribute__((address_space(1))) unsigned gu32;
constexpr long kSpinCap = 1L << 22;  // ~ tens of ms of polling at s_sleep 1: a hang becomes an error word

struct Sync {          // one memset block (zeroed before every launch), 16-byte multiple, at the allocation's start
  unsigned census;     // workgroups through the census
  unsigned top;        // leader arrivals (hierarchical) / all arrivals (flat)
  unsigned gen_flat;   // flat barrier generation
  unsigned err;        // timeout word
  unsigned members[8]; // workgroups per XCC
  unsigned xcnt[8 * 16];  // per-XCC arrival counters, one 64-byte line each
  unsigned xgen[8 * 16];  // per-XCC generation words, one 64-byte line each
};

__device__ __forceinline__ unsigned ld_rlx(unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(unsigned* p, unsigned v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_rlx(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// poll until *p >= target (monotonic counters / generations); false on timeout (error word set)
__device__ __forceinline__ bool wait_ge(unsigned* p, unsigned target, Sync* s) {
  for (long spins = 0; ld_rlx(p) < target; ++spins) {
    __builtin_amdgcn_s_sleep(1);
    if (spins > kSpinCap) {
      st_rlx(&s->err, 1u);
      return false;
    }
    if (ld_rlx(&s->err)) return false;
  }
  return true;
}
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v & 7u;
}
// publish: every storing wave drains its stores before the workgroup barrier that precedes the arrival
__device__ __forceinline__ void drain_and_sync() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}
__device__ __forceinline__ void acquire_and_sync() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// census: XCC membership; then every workgroup waits for the whole grid (flat, once per launch)
__device__ void census(Sync* s, unsigned nwg, unsigned& xcc, unsigned& nx) {
  __shared__ unsigned sh[2];
  if (threadIdx.x == 0) {
    xcc = xcc_id();
    add_rlx(&s->members[xcc], 1u);
    add_rlx(&s->census, 1u);
    wait_ge(&s->census, nwg, s);
    unsigned n = 0;
    for (int x = 0; x < 8; ++x) n += ld_rlx(&s->members[x]) ? 1u : 0u;
    sh[0] = xcc;
    sh[1] = n;
  }
  __syncthreads();
  xcc = sh[0];
  nx = sh[1];
}

__device__ __forceinline__ void barrier_flat(Sync* s, unsigned nwg, unsigned epoch) {
  drain_and_sync();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    add_rlx(&s->top, 1u);
    wait_ge(&s->top, nwg * epoch, s);
  }
  acquire_and_sync();
}

__device__ __forceinline__ void barrier_xcd(Sync* s, unsigned xcc, unsigned nx, unsigned epoch) {
  drain_and_sync();
  if (threadIdx.x == 0) {
    const unsigned mem = ld_rlx(&s->members[xcc]);
    const unsigned old = add_rlx(&s->xcnt[xcc * 16], 1u);
    if (old + 1 == mem * epoch) {  // this XCC's last arriver: its leader for this phase
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the XCC's L2 written back once
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      add_rlx(&s->top, 1u);
      wait_ge(&s->top, nx * epoch, s);
      st_rlx(&s->xgen[xcc * 16], epoch);
    } else {
      wait_ge(&s->xgen[xcc * 16], epoch, s);
    }
  }
  acquire_and_sync();
}

__device__ __forceinline__ void phase_body(const float* in, float* out, int W, int wg, int nwg, int nb) {
  const float* a = in + (long)wg * W;
  const float* b = in + (long)((wg + nb) % nwg) * W;
  float* o = out + (long)wg * W;
  for (int i = threadIdx.x * 4; i < W; i += blockDim.x * 4) {
    const float4 x = *reinterpret_cast<const float4*>(a + i), y = *reinterpret_cast<const float4*>(b + i);
    *reinterpret_cast<float4*>(o + i) = make_float4(0.5f * x.x + 0.25f * y.x + 1.f, 0.5f * x.y + 0.25f * y.y,
                                                    0.5f * x.z + 0.25f * y.z, 0.5f * x.w + 0.25f * y.w + 1.f);
  }
}

__global__ void step_kernel(const float* in, float* out, int W, int nb) {
  phase_body(in, out, W, blockIdx.x, gridDim.x, nb);
}

template <bool XCD>
__global__ __launch_bounds__(256) void persistent_kernel(float* b0, float* b1, int W, int P, Sync* s, int nb) {
  unsigned xcc, nx;
  census(s, gridDim.x, xcc, nx);
  for (int p = 0; p < P; ++p) {
    if (ld_rlx(&s->err)) return;  // a timed-out barrier: every workgroup leaves (wrong data, no hang)
    const float* in = (p & 1) ? b1 : b0;
    float* out = (p & 1) ? b0 : b1;
    phase_body(in, out, W, blockIdx.x, gridDim.x, nb);
    if (XCD) barrier_xcd(s, xcc, nx, (unsigned)p + 1);
    else barrier_flat(s, gridDim.x, (unsigned)p + 1);
  }
}

int main() {
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int P = 200;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  Sync* s;
  CK(hipMalloc(&s, sizeof(Sync)));
  printf("CUs %d, 256-thread workgroups, %d phases, sizeof(Sync) %zu\n", ncu, P, sizeof(Sync));
  int bad = 0;
  for (int per_cu : {1, 2}) {
    const int nwg = ncu * per_cu;
    for (int W : {1024, 16384}) {  // 4 KB or 64 KB per workgroup per phase
      const size_t n = (size_t)nwg * W, bytes = n * sizeof(float);
      std::vector<float> init(n), ref(n), got(n);
      for (size_t i = 0; i < n; ++i) init[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
      float *b0, *b1;
      CK(hipMalloc(&b0, bytes));
      CK(hipMalloc(&b1, bytes));
      for (int nb : {1, 8}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
        for (int p = 0; p < P; ++p) step_kernel<<<nwg, 256, 0, st>>>((p & 1) ? b1 : b0, (p & 1) ? b0 : b1, W, nb);
        CK(hipStreamEndCapture(st, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        float ms_g = 0.f;
        for (int rep = 0; rep < 2; ++rep) {
          CK(hipMemcpy(b0, init.data(), bytes, hipMemcpyHostToDevice));
          CK(hipEventRecord(e0, st));
          CK(hipGraphLaunch(ge, st));
          CK(hipEventRecord(e1, st));
          CK(hipStreamSynchronize(st));
          CK(hipEventElapsedTime(&ms_g, e0, e1));
        }
        CK(hipMemcpy(ref.data(), (P & 1) ? b1 : b0, bytes, hipMemcpyDeviceToHost));
        float ms[2] = {0.f, 0.f};
        unsigned herr[2] = {0, 0};
        bool same[2] = {true, true};
        for (int xcd = 0; xcd < 2; ++xcd) {
          for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemcpy(b0, init.data(), bytes, hipMemcpyHostToDevice));
            CK(hipMemsetAsync(s, 0, sizeof(Sync), st));
            CK(hipEventRecord(e0, st));
            if (xcd) persistent_kernel<true><<<nwg, 256, 0, st>>>(b0, b1, W, P, s, nb);
            else persistent_kernel<false><<<nwg, 256, 0, st>>>(b0, b1, W, P, s, nb);
            CK(hipEventRecord(e1, st));
            CK(hipStreamSynchronize(st));
            CK(hipEventElapsedTime(&ms[xcd], e0, e1));
            CK(hipMemcpy(&herr[xcd], &s->err, 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(got.data(), (P & 1) ? b1 : b0, bytes, hipMemcpyDeviceToHost));
            same[xcd] = same[xcd] && memcmp(got.data(), ref.data(), bytes) == 0;
          }
        }
        printf("%d WG/CU, W %5d floats/wg, neighbour +%d: graph of %d launches %.2f us/phase | persistent, flat "
               "barrier %.2f us/phase%s%s | persistent, XCD barrier %.2f us/phase%s%s\n",
               per_cu, W, nb, P, ms_g * 1e3f / P, ms[0] * 1e3f / P, herr[0] ? " TIMEOUT" : "",
               same[0] ? "" : " MISMATCH", ms[1] * 1e3f / P, herr[1] ? " TIMEOUT" : "", same[1] ? "" : " MISMATCH");
        bad |= herr[0] | herr[1] | !same[0] | !same[1];
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
      }
      CK(hipFree(b0));
      CK(hipFree(b1));
    }
  }
  CK(hipFree(s));
  printf(bad ? "FAILED\n" : "all persistent results bitwise equal to the launch chain\n");
  return bad;
}
