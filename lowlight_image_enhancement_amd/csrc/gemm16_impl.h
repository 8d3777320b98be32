// 16-bit MFMA GEMM kernels and their launchers (shared by gemm_bf16.hip and conv16.hip; every translation unit
// gets its own internal-linkage copy of the templates it instantiates, so the two compile in parallel).
#pragma once
// bf16-operand MFMA GEMM (perf mode): C = A(M,K) . W(N,K)^T with fp32 accumulation, v_mfma_f32_32x32x16_bf16.
// The reference trains under AMP (image_restoration_model.py:255, GradScaler :104-106): its convs take half-precision
// operands; here the operands are bf16 (no loss scaling needed: 8-bit exponent), accumulation and epilogue fp32.
// A may be stored fp32 (converted in the tile loader) or bf16; C/R/pre fp32 or bf16.  Same A/C modes as gemm.hip
// (space-to-depth gather for the down conv / up-conv dgrad, per-image column scale for SCA, depth-to-space scatter
// + residual for the up conv).  Weights come from a per-step bf16 copy of the flat parameter buffer; dgrads use
// the transposed copy so every launch is NT.
#include <hip/hip_bf16.h>
#include <stdlib.h>

#include "nbp_common.h"

using namespace nbp;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

// A modes: plain rows, space-to-depth gather, per-(image, column) scale, and 3x3 neighbourhood gather (implicit GEMM
// of a zero-padded 3x3 conv over an NHWC map: row m = pixel, k = tap * Cin + c with gh = H, gw = W, cs = Cin).
// C modes: plain, depth-to-space scatter, bias + ReLU, ReLU-mask by R (C = acc where R > 0, else 0), SimpleGate
// forward (C = t with channel pairs (c, C+c) interleaved, and pre <- g = t[2c] * t[2c+1]) and SimpleGate backward
// (acc = dg for column c; with R = t interleaved: C[2c] = dg * t[2c+1], C[2c+1] = dg * t[2c], row stride ldc).
enum { AM_PLAIN = 0, AM_S2D = 1, AM_SCALE = 2, AM_IM2COL = 3, AM_CONV = 4 };
enum { CM_PLAIN = 0, CM_D2S = 1, CM_RELU = 2, CM_MASK = 3, CM_SG = 4, CM_SGBWD = 5, CM_LNBWD = 6, CM_RESLN = 7,
       CM_CHANDOT = 8, CM_SGBWD_RC = 9, CM_FFN = 10 };

struct GemmPB {
  const void* A;
  long lda;
  const float* a_scale;
  int rows_per_img;
  const void* B;  // 16-bit weights (the kernel's operand type H)
  long ldb;
  void* C;
  long ldc;
  int M, N, K;
  int gh, gw, cs;
  const float* bias;
  const void* R;
  const float* rscale;
  void* pre;
  // CM_RESLN (tiled, N == BN == 128): the LayerNorm2d forward of each stored C row in the epilogue
  const float* lnw;
  const float* lnb;
  void* nout;
  float2* stats;
  float eps;
  // CM_LNBWD (tiled, N == BN == 128): R = the LN input x, stats_in = (mu, den), lnw, dres; LN weight / bias gradient
  // partials per 64-row tile into slab_w / slab_b [M / 64][N]
  const float2* stats_in;
  const void* dres;
  float* slab_w;
  float* slab_b;
  // AM_CONV (general KH x KW / stride / zero-pad implicit GEMM): gh x gw = the output map, ih x iw = the input map,
  // k = (ki * kw + kj) * cs + c
  int kh, kw, stride, pad, ih, iw;
  // AM_IM2COL: the K-tiles lie inside one tap (Cin % 64 == 0): the DMA issue takes the tap per stage
  int tap_tile;
  // gemm_glds_kernel tile order: 0 = blockIdx.x -> M tile, blockIdx.y -> N tile (dispatch deals consecutive M tiles to
  // different XCDs); 1 = each XCD takes a contiguous run of M tiles with all their N tiles, so the 3x3 taps' row
  // overlaps between neighbouring M tiles (and the shared A panels) are L2 hits on one XCD
  int tile_map;
};

// Timeline probe (scripts/gemm_timeline.py; built only into the probe library, scripts/build_probe.py, never into the
// production .so): thread 0 of each gemm_glds_kernel workgroup records the 100 MHz global clock at 6 points of its life
// (slot 0: the first instruction; 1: the kernel arguments in registers; 2: prologue DMAs issued; 3: K-tile 0 landed;
// 4: last MFMA issued; 5: epilogue stores landed) plus HW_ID / XCC_ID (slots 6 / 7), 8 words per workgroup in grid
// order
#ifdef NBP_GEMM_PROBE
constexpr int GEMM_PROBE_WGS = 16384;
__device__ unsigned long long g_gemm_probe[GEMM_PROBE_WGS * 8];
__device__ __forceinline__ void gemm_stamp_at(int i, unsigned long long t) {
  if (threadIdx.x == 0) {
    const unsigned w = blockIdx.x + gridDim.x * blockIdx.y;
    if (w < GEMM_PROBE_WGS) {
      g_gemm_probe[w * 8 + i] = t;
      if (i == 0) {
        g_gemm_probe[w * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        g_gemm_probe[w * 8 + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
      }
    }
  }
}
#define GEMM_STAMP(i) gemm_stamp_at(i, __builtin_amdgcn_s_memrealtime())
#else
#define GEMM_STAMP(i) ((void)0)
#endif

__device__ __forceinline__ long s2d_off(int m, int k, int gh, int gw, int cs) {
  const int per = gh * gw;
  const int b = m / per, rem = m - b * per;
  const int i = rem / gw, j = rem - i * gw;
  const int q = k / cs, c = k - q * cs;
  const int kh = q >> 1, kw = q & 1;
  return ((long)(b * 2 * gh + 2 * i + kh) * (2 * gw) + 2 * j + kw) * cs + c;
}

template <typename T>
__device__ __forceinline__ float ldf(const void* p, long off) {
  return (float)reinterpret_cast<const T*>(p)[off];
}
template <typename T>
__device__ __forceinline__ void stf(void* p, long off, float v) {
  reinterpret_cast<T*>(p)[off] = (T)v;
}

// 8 consecutive elements of A at element offset `off`, optionally scaled, as the 16-bit operand type H
template <typename TA, int AMODE, typename H>
__device__ __forceinline__ vec_t<H, 8> load8(const void* A, long off, const float* scale) {
  vec_t<H, 8> r;
  if constexpr (sizeof(TA) == 4) {
    const float4 a = ld4(reinterpret_cast<const float*>(A) + off);
    const float4 b = ld4(reinterpret_cast<const float*>(A) + off + 4);
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    if (AMODE == AM_SCALE) {
      const float4 s0 = ld4(scale), s1 = ld4(scale + 4);
      v[0] *= s0.x; v[1] *= s0.y; v[2] *= s0.z; v[3] *= s0.w;
      v[4] *= s1.x; v[5] *= s1.y; v[6] *= s1.z; v[7] *= s1.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (H)v[j];
  } else {
    static_assert(sizeof(TA) == 2, "16-bit A is the operand type");
    r = *reinterpret_cast<const vec_t<H, 8>*>(reinterpret_cast<const H*>(A) + off);
    if (AMODE == AM_SCALE) {
      const float4 s0 = ld4(scale), s1 = ld4(scale + 4);
      const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = (H)((float)r[j] * s[j]);
    }
  }
  return r;
}

// 8 consecutive fp32 values <-> storage type (16 bytes of 16-bit / 32 bytes of fp32)
template <typename T>
__device__ __forceinline__ void ld8f(const void* base, long off, float* v) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = ld4(reinterpret_cast<const float*>(base) + off), b = ld4(reinterpret_cast<const float*>(base) + off + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const vec_t<T, 8> r = *reinterpret_cast<const vec_t<T, 8>*>(reinterpret_cast<const T*>(base) + off);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)r[j];
  }
}
template <typename T>
__device__ __forceinline__ void st8f(void* base, long off, const float* v) {
  if constexpr (sizeof(T) == 4) {
    float* d = reinterpret_cast<float*>(base) + off;
    st4(d, make_float4(v[0], v[1], v[2], v[3]));
    st4(d + 4, make_float4(v[4], v[5], v[6], v[7]));
  } else {
    vec_t<T, 8> r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (T)v[j];
    *reinterpret_cast<vec_t<T, 8>*>(reinterpret_cast<T*>(base) + off) = r;
  }
}

// Epilogue of the tiled kernels: the fp32 accumulators (4 waves in a 2x2 arrangement, each (BM/2) x (BN/2) of 32x32
// MFMA tiles) are staged through LDS (smem, aliasing the operand buffers; the caller has finished every read of them)
// so that bias / pre-activation / residual R + rscale * v / the C store all move 8 consecutive columns per thread.
// WM x WN waves (default 2 x 2), each (BM / WM) x (BN / WN) of 32 x 32 MFMA tiles; NT = 64 WM WN threads.
// PASSES > 1 (tiles whose fp32 image would not fit in LDS): the rows of wave-row group q (WM / PASSES wave rows) are
// staged and stored in pass q, one pass after the other through the same LDS rows.
// CM_LNBWD chunk inputs loaded before the K loop (gemm_glds_kernel, 16-bit C): the x / dres chunks and the row
// statistics of each of the thread's NPRE epilogue chunks (their latency then overlaps the K loop)
template <int NPRE>
struct LnPre {
  uint4 x[NPRE], r[NPRE];
  float2 st[NPRE];
};

template <int BM, int BN, int CMODE, typename TC, typename H, int WN = 2, int WM = 2, int PASSES = 1, int NPRE = 0>
__device__ __forceinline__ void gemm_epilogue(const GemmPB& p, floatx16 (&acc)[BM / (32 * WM)][BN / (32 * WN)],
                                              unsigned char* smem, int m0, int n0,
                                              const LnPre<(NPRE > 0 ? NPRE : 1)>* pre = nullptr) {
  constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN), NT = 64 * WM * WN;
  static_assert((WN == 2 && WM == 2) || (CMODE != CM_LNBWD && CMODE != CM_CHANDOT),
                "cross-wave reductions assume 2 x 2 waves");
  static_assert(PASSES == 1 || (WM % PASSES == 0 && CMODE != CM_LNBWD && CMODE != CM_CHANDOT && CMODE != CM_RESLN),
                "multi-pass epilogue: plain row-local modes");
  constexpr int CLS = BN + 4;  // fp32 C-tile row stride
  constexpr int PR = BM / PASSES;  // tile rows per pass
  float* Cs = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int M = p.M, N = p.N;
  constexpr int G8 = BN / 8;
  const bool vec = (N % 8 == 0) && (CMODE == CM_D2S || p.ldc % 8 == 0);
  // CM_CHANDOT (SCA backward, NAFNet_arch.py:39-41): besides C, per-column partial sums over the tile's rows of
  // C (bf16-rounded) * R (the SimpleGate output g) -> pre[image][tile within image][col] (fp32), the per-image channel
  // dot img_chan_dot computes, without re-reading C.  The launcher guarantees BM | rows_per_img.
  float cd[8], cb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cd[j] = cb[j] = 0.f;
  for (int pass = 0; pass < PASSES; ++pass) {
  if (pass) __syncthreads();  // the previous pass's rows are stored: the LDS rows are free
  if (PASSES == 1 || wm / (WM / PASSES) == pass) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * (BN / WN) + j * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * (BM / WM) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) - pass * PR;
          Cs[row * CLS + col] = acc[i][j][r];
        }
      }
  }
  __syncthreads();
  constexpr int NIT = (PR * G8 + NT - 1) / NT;
  static_assert(NPRE == 0 || (CMODE == CM_LNBWD && NPRE == NIT && PASSES == 1), "preloaded LN-backward chunks");
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + it * NT;
    if (e >= PR * G8) break;
    const int row = e / G8, c8 = (e % G8) * 8;
    const int grow = m0 + pass * PR + row, gcol = n0 + c8;
    if (grow >= M || gcol >= N) continue;
    float v[8];
    const float4 c0 = ld4(Cs + row * CLS + c8), c1 = ld4(Cs + row * CLS + c8 + 4);
    v[0] = c0.x; v[1] = c0.y; v[2] = c0.z; v[3] = c0.w; v[4] = c1.x; v[5] = c1.y; v[6] = c1.z; v[7] = c1.w;
    if constexpr (CMODE == CM_LNBWD) {  // dx = (g - yhat mean(g yhat) - mean(g)) / den + dres, g = dn * lnw
      static_assert(BN == 128 || BN == 256 || BN == 512, "CM_LNBWD (tiled): full-row tiles");
      const long off = (long)grow * N + gcol;
      float xv[8], rv[8];
      float2 st;
      if constexpr (NPRE > 0) {
        const vec_t<TC, 8> xr = __builtin_bit_cast(vec_t<TC, 8>, pre->x[it]);
        const vec_t<TC, 8> rr = __builtin_bit_cast(vec_t<TC, 8>, pre->r[it]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[j] = (float)xr[j];
          rv[j] = (float)rr[j];
        }
        st = pre->st[it];
      } else {
        ld8f<TC>(p.R, off, xv);
        ld8f<TC>(p.dres, off, rv);
        st = p.stats_in[grow];
      }
      const float inv = 1.f / st.y;
      const float4 w0 = ld4(p.lnw + gcol), w1 = ld4(p.lnw + gcol + 4);
      const float lw[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float yh[8], sg = 0.f, sgy = 0.f;
      // the arithmetic of ln_bwd_nhwc (and of nbp_ffn_rows_bwd), contractions spelt out: the same dx bits whichever
      // kernel runs the LayerNorm backward
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        yh[j] = (xv[j] - st.x) * inv;
        sg = fmaf(v[j], lw[j], sg);
        sgy = fmaf(v[j] * lw[j], yh[j], sgy);
        cd[j] = fmaf(v[j], yh[j], cd[j]);  // dlnw partial
        cb[j] += v[j];                      // dlnb partial
      }
      sg = group_sum<G8>(sg);
      sgy = group_sum<G8>(sgy);
      const float mg = sg / (float)N, mgy = sgy / (float)N;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = fmaf(inv, fmaf(-yh[j], mgy, v[j] * lw[j]) - mg, rv[j]);
        asm volatile("" : "+v"(o[j]));  // rounded to fp32, then to the storage type
      }
      st8f<TC>(p.C, off, o);
      continue;
    }
    if constexpr (CMODE == CM_CHANDOT) {
      const long off = (long)grow * p.ldc + gcol;
      float gv[8];
      ld8f<TC>(p.R, off, gv);
      vec_t<H, 8> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (H)v[j];
        cd[j] = fmaf((float)o[j], gv[j], cd[j]);
      }
      *reinterpret_cast<vec_t<H, 8>*>(reinterpret_cast<H*>(p.C) + off) = o;
      continue;
    }
    if (CMODE == CM_SGBWD) {
      // 8 gate channels -> 16 interleaved (t, dt) values
      const long off = (long)grow * p.ldc + 2 * gcol;
      if (vec) {
        float ta[8], tb[8], oa[8], ob[8];
        ld8f<TC>(p.R, off, ta);
        ld8f<TC>(p.R, off + 8, tb);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // fp32 products, then one rounding each (the SimpleGate convention)
          oa[2 * j] = v[j] * ta[2 * j + 1];
          oa[2 * j + 1] = v[j] * ta[2 * j];
          ob[2 * j] = v[4 + j] * tb[2 * j + 1];
          ob[2 * j + 1] = v[4 + j] * tb[2 * j];
          asm volatile("" : "+v"(oa[2 * j]), "+v"(oa[2 * j + 1]), "+v"(ob[2 * j]), "+v"(ob[2 * j + 1]));
        }
        st8f<TC>(p.C, off, oa);
        st8f<TC>(p.C, off + 8, ob);
      } else {
        for (int j = 0; j < 8 && gcol + j < N; ++j) {
          const float t0 = ldf<TC>(p.R, off + 2 * j), t1 = ldf<TC>(p.R, off + 2 * j + 1);
          float q0 = v[j] * t1, q1 = v[j] * t0;
          asm volatile("" : "+v"(q0), "+v"(q1));
          stf<TC>(p.C, off + 2 * j, q0);
          stf<TC>(p.C, off + 2 * j + 1, q1);
        }
      }
      continue;
    }
    if (vec) {
      const long off = CMODE == CM_D2S ? s2d_off(grow, gcol, p.gh, p.gw, p.cs) : (long)grow * p.ldc + gcol;
      if (p.bias) {
        const float4 b0 = ld4(p.bias + gcol), b1 = ld4(p.bias + gcol + 4);
        v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w; v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
      }
      if (CMODE == CM_RELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
      } else if (CMODE == CM_MASK) {
        float rv[8];
        ld8f<TC>(p.R, off, rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = rv[j] > 0.f ? v[j] : 0.f;
      }
      if (CMODE == CM_SG) {
        // an fp32 product, then one rounding to the storage type -- the SimpleGate convention of every other kernel
        // (left implicit, the fp16 build formed two of a chunk's four gates with v_fma_mixlo_f16, a single rounding of
        // the exact product, and the other two with v_pk_mul_f32 + v_cvt_pk_f16_f32)
        float g[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          g[j] = v[2 * j] * v[2 * j + 1];
          asm volatile("" : "+v"(g[j]));
        }
        // 4 gate values (8 bytes of bf16 / 16 of fp32) at row grow, column gcol / 2 of the [M][N/2] map
        if constexpr (sizeof(TC) == 4) {
          st4(reinterpret_cast<float*>(p.pre) + (long)grow * (p.ldc / 2) + gcol / 2, make_float4(g[0], g[1], g[2], g[3]));
        } else {
          vec_t<H, 4> o;
          o[0] = (H)g[0]; o[1] = (H)g[1]; o[2] = (H)g[2]; o[3] = (H)g[3];
          *reinterpret_cast<vec_t<H, 4>*>(reinterpret_cast<H*>(p.pre) + (long)grow * (p.ldc / 2) + gcol / 2) = o;
        }
      } else if (p.pre) {
        st8f<TC>(p.pre, off, v);
      }
      if (CMODE != CM_MASK && p.R) {
        float rv[8];
        ld8f<TC>(p.R, off, rv);
        if (p.rscale) {
          const float4 s0 = ld4(p.rscale + gcol), s1 = ld4(p.rscale + gcol + 4);
          const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          // one fused multiply-add, spelt out (what the compiler contracted r + s * v to; left implicit, a change of
          // the code around it -- a residual preload tried in round 4 -- un-fused it and changed the stored bits)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = fmaf(sc[j], v[j], rv[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = rv[j] + v[j];
        }
      }
      st8f<TC>(p.C, off, v);
      if constexpr (CMODE == CM_RESLN) {  // the row's G8 chunks are G8 consecutive lanes (BN = N): group sums
        static_assert(BN == 128 || BN == 256 || BN == 512, "CM_RESLN (tiled): full-row tiles");
        float xv[8], sm = 0.f, q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[j] = (float)(H)v[j];
          sm += xv[j];
        }
        sm = group_sum<G8>(sm);
        const float mu = sm / (float)N;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = xv[j] - mu;
          q = fmaf(d, d, q);
        }
        q = group_sum<G8>(q);
        const float dd = sqrtf(q / (float)N + p.eps), inv = 1.f / dd;
        const float4 w0 = ld4(p.lnw + gcol), w1 = ld4(p.lnw + gcol + 4), b0 = ld4(p.lnb + gcol), b1 = ld4(p.lnb + gcol + 4);
        const float lw[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        const float lb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaf(lw[j], (xv[j] - mu) * inv, lb[j]);
        st8f<TC>(p.nout, (long)grow * N + gcol, o);
        if (gcol == 0) p.stats[grow] = make_float2(mu, dd);
      }
    } else {
      for (int j = 0; j < 8 && gcol + j < N; ++j) {
        const int col = gcol + j;
        const long off = CMODE == CM_D2S ? s2d_off(grow, col, p.gh, p.gw, p.cs) : (long)grow * p.ldc + col;
        float x = v[j] + (p.bias ? p.bias[col] : 0.f);
        if (CMODE == CM_RELU) x = fmaxf(x, 0.f);
        if (CMODE == CM_MASK) x = ldf<TC>(p.R, off) > 0.f ? x : 0.f;
        if (CMODE == CM_SG) {
          v[j] = x;
          if (j & 1) {
            float gq = v[j - 1] * x;
            asm volatile("" : "+v"(gq));  // (as the vector path: an fp32 product, then one rounding)
            stf<TC>(p.pre, (long)grow * (p.ldc / 2) + col / 2, gq);
          }
        } else if (p.pre) {
          stf<TC>(p.pre, off, x);
        }
        if (CMODE != CM_MASK && p.R) x = ldf<TC>(p.R, off) + (p.rscale ? p.rscale[col] : 1.f) * x;
        stf<TC>(p.C, off, x);
      }
    }
  }
  }  // pass
  if constexpr (CMODE == CM_LNBWD) {  // threads sharing a column chunk: lanes G8 apart, then the 4 waves (fixed order)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int o = G8; o < 64; o <<= 1) {
        cd[j] += __shfl_xor(cd[j], o, 64);
        cb[j] += __shfl_xor(cb[j], o, 64);
      }
    __syncthreads();
    if (lane < G8)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        Cs[(wave * 2 + 0) * BN + lane * 8 + j] = cd[j];
        Cs[(wave * 2 + 1) * BN + lane * 8 + j] = cb[j];
      }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {  // (BN 512: two columns per thread)
      const float tw = ((Cs[0 * BN + c] + Cs[2 * BN + c]) + Cs[4 * BN + c]) + Cs[6 * BN + c];
      const float tb = ((Cs[1 * BN + c] + Cs[3 * BN + c]) + Cs[5 * BN + c]) + Cs[7 * BN + c];
      p.slab_w[(long)(m0 / BM) * N + c] = tw;  // the tile's row block (not blockIdx: tile_map may permute it)
      p.slab_b[(long)(m0 / BM) * N + c] = tb;
    }
  }
  if constexpr (CMODE == CM_CHANDOT) {  // threads sharing a column chunk: lanes 8 apart, then the 4 waves (fixed order)
    static_assert(G8 == 8 && BM == 64, "CM_CHANDOT: 64 x 64 tiles");
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      cd[j] += __shfl_xor(cd[j], 8, 64);
      cd[j] += __shfl_xor(cd[j], 16, 64);
      cd[j] += __shfl_xor(cd[j], 32, 64);
    }
    __syncthreads();
    if (lane < 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) Cs[wave * 64 + lane * 8 + j] = cd[j];
    __syncthreads();
    if (tid < 64 && n0 + tid < N) {
      const int img = m0 / p.rows_per_img, chunk = (m0 - img * p.rows_per_img) / BM, chunks = p.rows_per_img / BM;
      const float t = ((Cs[tid] + Cs[64 + tid]) + Cs[128 + tid]) + Cs[192 + tid];
      reinterpret_cast<float*>(p.pre)[((long)img * chunks + chunk) * N + n0 + tid] = t;
    }
  }
}

// Register-staged tiled kernel (any A type / mode): 4 waves in a 2x2 arrangement, each (BM/2) x (BN/2) of 32x32 MFMA
// tiles.  K-loop: BK-wide tiles, double-buffered LDS (one barrier per K step; the next tile's global loads are in
// flight during the current tile's MFMAs).  Epilogue: gemm_epilogue.
template <int BM, int BN, int BK, int AMODE, int CMODE, typename TA, typename TC, typename H>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(GemmPB p) {
  static_assert(sizeof(TA) == 4 || sizeof(TA) == sizeof(H), "A is fp32 or the operand type");
  static_assert(sizeof(TC) == 4 || sizeof(TC) == sizeof(H), "C is fp32 or the operand type");
  constexpr int LS = BK + 8;  // 80 / 144-byte LDS rows: conflict-free 16-byte fragment reads
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int KC = BK / 8;  // 8-element chunks per tile row
  constexpr int A_IT = BM * KC / 256, B_IT = BN * KC / 256;
  constexpr int AB_BYTES = 2 * (BM + BN) * LS * 2;
  constexpr int CLS = BN + 4;  // fp32 C-tile row stride
  constexpr int C_BYTES = BM * CLS * 4;
  constexpr int SM_BYTES = AB_BYTES > C_BYTES ? AB_BYTES : C_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM_BYTES];
  H* As = reinterpret_cast<H*>(smem);       // [2][BM][LS]
  H* Bs = As + 2 * BM * LS;                       // [2][BN][LS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int M = p.M, N = p.N, K = p.K;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // two register sets: with BK = 64 the loads of K-tiles t+1 and t+2 are in flight while tile t is multiplied
  vec_t<H, 8> ra0[A_IT], rb0[B_IT], ra1[A_IT], rb1[B_IT];
  auto load_tiles = [&](int k0, vec_t<H, 8>* ra, vec_t<H, 8>* rb) {
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int idx = tid + it * 256;
      const int r = idx / KC, kc = idx % KC;
      const int m = m0 + r, k = k0 + kc * 8;
      vec_t<H, 8> v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
      if (AMODE == AM_CONV) {
        if (m < M && k < K) {
          const int per = p.gh * p.gw, b = m / per, rem = m - b * per, oi = rem / p.gw, oj = rem - oi * p.gw;
          const int t = k / p.cs, c = k - t * p.cs, ki = t / p.kw, kj = t - ki * p.kw;
          const int ii = oi * p.stride + ki - p.pad, jj = oj * p.stride + kj - p.pad;
          if (ii >= 0 && ii < p.ih && jj >= 0 && jj < p.iw)
            v = load8<TA, AM_PLAIN, H>(p.A, ((long)(b * p.ih + ii) * p.iw + jj) * p.cs + c, nullptr);
        }
      } else if (AMODE == AM_IM2COL) {
        if (m < M && k < K) {
          const int per = p.gh * p.gw, b = m / per, rem = m - b * per, i = rem / p.gw, j = rem - i * p.gw;
          const int t = k / p.cs, c = k - t * p.cs;
          const int ii = i + t / 3 - 1, jj = j + t % 3 - 1;
          if (ii >= 0 && ii < p.gh && jj >= 0 && jj < p.gw)
            v = load8<TA, AM_PLAIN, H>(p.A, ((long)(b * p.gh + ii) * p.gw + jj) * p.cs + c, nullptr);
        }
      } else if (m < M && k < K) {
        long off;
        if (AMODE == AM_S2D) off = s2d_off(m, k, p.gh, p.gw, p.cs);
        else off = (long)m * p.lda + k;
        const float* sc = AMODE == AM_SCALE ? p.a_scale + (long)(m / p.rows_per_img) * K + k : nullptr;
        v = load8<TA, AMODE, H>(p.A, off, sc);
      }
      ra[it] = v;
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int idx = tid + it * 256;
      const int r = idx / KC, kc = idx % KC;
      const int n = n0 + r, k = k0 + kc * 8;
      vec_t<H, 8> v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
      if (n < N && k < K) v = *reinterpret_cast<const vec_t<H, 8>*>(reinterpret_cast<const H*>(p.B) + (long)n * p.ldb + k);
      rb[it] = v;
    }
  };
  auto store_tiles = [&](int buf, const vec_t<H, 8>* ra, const vec_t<H, 8>* rb) {
    H* a = As + buf * BM * LS;
    H* b = Bs + buf * BN * LS;
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int idx = tid + it * 256;
      *reinterpret_cast<vec_t<H, 8>*>(a + (idx / KC) * LS + (idx % KC) * 8) = ra[it];
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int idx = tid + it * 256;
      *reinterpret_cast<vec_t<H, 8>*>(b + (idx / KC) * LS + (idx % KC) * 8) = rb[it];
    }
  };
  const int arow = wm * (BM / 2) + (lane & 31);
  const int brow = wn * (BN / 2) + (lane & 31);
  const int kh = (lane >> 5) * 8;
  auto compute = [&](int buf) {
    const H* a_s = As + buf * BM * LS;
    const H* b_s = Bs + buf * BN * LS;
#pragma unroll
    for (int s = 0; s < BK; s += 16) {
      vec_t<H, 8> a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const vec_t<H, 8>*>(a_s + (arow + i * 32) * LS + s + kh);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const vec_t<H, 8>*>(b_s + (brow + j * 32) * LS + s + kh);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x16(a[i], b[j], acc[i][j]);
    }
  };

  const int nk = (K + BK - 1) / BK;
  if constexpr (BK == 32) {
    // short K (one or two tiles): one register set, the next tile's loads in flight during the MFMAs
    load_tiles(0, ra0, rb0);
    store_tiles(0, ra0, rb0);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      const int buf = t & 1;
      if (t + 1 < nk) load_tiles((t + 1) * BK, ra0, rb0);
      compute(buf);
      if (t + 1 < nk) store_tiles(buf ^ 1, ra0, rb0);
      __syncthreads();
    }
  } else {
    load_tiles(0, ra0, rb0);
    store_tiles(0, ra0, rb0);
    if (nk > 1) load_tiles(BK, ra1, rb1);
    if (nk > 2) load_tiles(2 * BK, ra0, rb0);
    __syncthreads();
    // steady state, unrolled by two so each register set is addressed statically:
    //   even step t: tile t in LDS buf 0, t+1 in set 1, t+2 in flight in set 0
    //   odd step t+1: tile t+1 in LDS buf 1, t+2 in set 0, t+3 in flight in set 1
    for (int t = 0; t < nk; t += 2) {
      compute(0);
      if (t + 1 < nk) {
        store_tiles(1, ra1, rb1);
        if (t + 3 < nk) load_tiles((t + 3) * BK, ra1, rb1);
      }
      __syncthreads();
      if (t + 1 >= nk) break;
      compute(1);
      if (t + 2 < nk) {
        store_tiles(0, ra0, rb0);
        if (t + 4 < nk) load_tiles((t + 4) * BK, ra0, rb0);
      }
      __syncthreads();
    }
  }

  gemm_epilogue<BM, BN, CMODE, TC, H>(p, acc, smem, m0, n0);
}

// ---------------------------------------------------------------- LDS-DMA tiled kernel (16-bit A)
// Same tiles, fragment order and MFMA sequence as gemm_bf16_kernel (so the same accumulation order: results are
// bitwise those of the register-staged kernel), but the operand tiles go global -> LDS with global_load_lds_dwordx4
// (no VGPR staging, no ds_write pass) into an NS-deep ring: NS - 1 K-tiles are in flight while one is multiplied,
// retired by a counted vmcnt and a raw s_barrier (a __syncthreads would drain the ring: vmcnt(0)).
// Per stage: A [BM][64] then B [BN][64] of 128-byte rows, the 16-byte chunk c of row r at slot c ^ ((r >> 1) & 7)
// (a glds instruction writes 1 KB lane-linearly, so the permutation is applied to each lane's SOURCE address; the
// fragment reads, lanes 0..31 on rows r..r+31 at one chunk, then hit 16 distinct slots per ds_read_b128 lane group),
// then for AM_SCALE the tile's 64 fp32 column scales (one 4-byte glds).  Out-of-range rows / columns / K tail and the
// zero padding of AM_IM2COL read g_zero16 (LDS-DMA helpers: nbp_common.h).
// BK = 32 (plain / im2col A): 64-byte rows, chunk c of row r at slot c ^ ((r >> 2) & 3) (again 16 distinct slots per
// ds_read_b128 lane group); half the bytes per stage, so twice the ring depth fits in the same LDS -- the 256 x 256
// tiles keep 3-4 K-tiles in flight instead of one.  The MFMA sequence per output element does not depend on BK.
template <int BM, int BN, int NS, int AMODE, int CMODE, typename TC, typename H, int WN = 2, int WM = 2, int BK = 64>
__global__ __launch_bounds__(64 * WM * WN) void gemm_glds_kernel(GemmPB p) {
  constexpr int NW = WM * WN;  // waves: WM along M x WN along N
  constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);
  static_assert(TM >= 1 && TN >= 1, "tile too small for the wave layout");
  static_assert(BK == 64 || (BK == 32 && AMODE != AM_SCALE), "K-tile width");
  constexpr int RB = 2 * BK, CPR = RB / 16, RPI = 1024 / RB;  // row bytes, 16-B chunks per row, rows per glds
  constexpr int A_BYTES = BM * RB, B_BYTES = BN * RB;
  constexpr int SC_BYTES = AMODE == AM_SCALE ? 256 : 0;
  constexpr int ST_BYTES = A_BYTES + B_BYTES + SC_BYTES;
  constexpr int GA = BM / (RPI * NW), GB = BN / (RPI * NW);  // 1-KB glds instructions per wave per stage
  static_assert(GA * RPI * NW == BM && GB * RPI * NW == BN, "DMA rows per wave");
  constexpr int G = GA + GB + (AMODE == AM_SCALE ? 1 : 0);
  // epilogue passes: BK 64: 1 while the whole fp32 tile image fits in LDS, else one per wave row (256 x 256 tiles);
  // BK 32: the fewest passes whose rows fit in the operand ring (the epilogue never sets the workgroup's LDS size)
  constexpr int CF = BM * (BN + 4) * 4, RING = NS * ST_BYTES;
  constexpr int EPP = BK == 64 ? (CF <= 160 * 1024 ? 1 : WM)
                               : (CF <= RING ? 1 : (WM % 2 == 0 && CF / 2 <= RING ? 2 : (WM % 4 == 0 && CF / 4 <= RING ? 4 : WM)));
  constexpr int C_BYTES = BM / EPP * (BN + 4) * 4;
  constexpr int SM_BYTES = NS * ST_BYTES > C_BYTES ? NS * ST_BYTES : C_BYTES;
  static_assert(NS >= 2 && NS <= 5, "ring depth");
  static_assert(SM_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM_BYTES];
#ifdef NBP_GEMM_PROBE
  const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
  {
    int mk = p.M + p.K;  // the kernel arguments in registers
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(mk)::"memory");
    const unsigned long long t_args = __builtin_amdgcn_s_memrealtime() + (mk == -7 ? 1 : 0);
    gemm_stamp_at(0, t_entry);
    gemm_stamp_at(1, t_args);
  }
#endif
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // slot permutation key of row r
  auto swz = [](int r) { return BK == 64 ? (r >> 1) & 7 : (r >> 2) & 3; };
  int bx = blockIdx.x, by = blockIdx.y;
  if (p.tile_map) {
    const int L = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    bx = L / gridDim.y;
    by = L - bx * gridDim.y;
  }
  const int m0 = bx * BM, n0 = by * BN;
  const int M = p.M, N = p.N, K = p.K;
  const H* A = reinterpret_cast<const H*>(p.A);
  const H* B = reinterpret_cast<const H*>(p.B);
  const int lr = lane / CPR, lc = lane % CPR;

  // this lane's source rows: instruction i covers tile rows (wave * GA + i) * RPI .. + RPI - 1, the lane row lr, chunk
  // slot lc
  int a_m[GA], a_kof[GA], a_b[GA], a_i[GA], a_j[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int r = (wave * GA + i) * RPI + lr;
    a_m[i] = m0 + r;
    a_kof[i] = 8 * (lc ^ swz(r));
    a_b[i] = a_i[i] = a_j[i] = 0;
    if constexpr (AMODE == AM_S2D || AMODE == AM_IM2COL) {
      const int per = p.gh * p.gw, m = a_m[i] < M ? a_m[i] : 0;
      a_b[i] = m / per;
      const int rem = m - a_b[i] * per;
      a_i[i] = rem / p.gw;
      a_j[i] = rem - a_i[i] * p.gw;
    }
  }
  int b_n[GB], b_kof[GB];
#pragma unroll
  for (int i = 0; i < GB; ++i) {
    const int r = (wave * GB + i) * RPI + lr;
    b_n[i] = n0 + r;
    b_kof[i] = 8 * (lc ^ swz(r));
  }
  const float* sc_row = AMODE == AM_SCALE ? p.a_scale + (long)(m0 / p.rows_per_img) * K : nullptr;
  // the zero page's address in registers (laundered through asm: otherwise re-loaded from the GOT at every use)
  const void* zp = g_zero16;
  asm volatile("" : "+s"(zp));

  const int nk = (K + BK - 1) / BK;
  // IM2COL with Cin a multiple of BK: a K-tile lies inside one tap, so the tap (and its pixel offset) is per stage, not
  // per lane -- no per-lane integer division in the DMA issue
  const bool tap_tile = AMODE == AM_IM2COL && p.tap_tile != 0;
  auto issue = [&](int t) {
    unsigned char* st = smem + (t % NS) * ST_BYTES;
    const int k0 = t * BK;
    int tap_off = 0, tap_c0 = 0, tap_di = 0, tap_dj = 0;
    if (AMODE == AM_IM2COL && tap_tile) {
      const int t9 = k0 / p.cs;
      tap_c0 = k0 - t9 * p.cs;
      tap_di = t9 / 3 - 1;
      tap_dj = t9 % 3 - 1;
      tap_off = tap_di * p.gw + tap_dj;
    }
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      const int k = k0 + a_kof[i];
      const void* src = zp;
      if (AMODE == AM_IM2COL && tap_tile) {
        const int ii = a_i[i] + tap_di, jj = a_j[i] + tap_dj;
        if (a_m[i] < M && k < K && ii >= 0 && ii < p.gh && jj >= 0 && jj < p.gw)
          src = A + ((long)a_m[i] + tap_off) * p.cs + tap_c0 + a_kof[i];
      } else if (a_m[i] < M && k < K) {
        if constexpr (AMODE == AM_S2D) {
          const int q = k / p.cs, c = k - q * p.cs;
          src = A + ((long)(a_b[i] * 2 * p.gh + 2 * a_i[i] + (q >> 1)) * (2 * p.gw) + 2 * a_j[i] + (q & 1)) * p.cs + c;
        } else if constexpr (AMODE == AM_IM2COL) {
          const int t9 = k / p.cs, c = k - t9 * p.cs;
          const int ii = a_i[i] + t9 / 3 - 1, jj = a_j[i] + t9 % 3 - 1;
          if (ii >= 0 && ii < p.gh && jj >= 0 && jj < p.gw)
            src = A + ((long)(a_b[i] * p.gh + ii) * p.gw + jj) * p.cs + c;
        } else {
          src = A + (long)a_m[i] * p.lda + k;
        }
      }
      glds16(src, st + (wave * GA + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < GB; ++i) {
      const int k = k0 + b_kof[i];
      const void* src = (b_n[i] < N && k < K) ? (const void*)(B + (long)b_n[i] * p.ldb + k) : zp;
      glds16(src, st + A_BYTES + (wave * GB + i) * 1024);
    }
    if constexpr (AMODE == AM_SCALE) {  // every wave loads the same 64 scales (identical bytes, one instruction each)
      const int k = k0 + lane;
      glds4(k < K ? (const void*)(sc_row + k) : zp, st + A_BYTES + B_BYTES);
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int key = swz(lane & 31);  // the key of every fragment row: rows are 32-aligned + (lane & 31)
  auto compute = [&](int buf) {
    const unsigned char* a_s = smem + buf * ST_BYTES;
    const unsigned char* b_s = a_s + A_BYTES;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int slot = ((2 * s + (lane >> 5)) ^ key) << 4;
      vec_t<H, 8> a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[i] = *reinterpret_cast<const vec_t<H, 8>*>(a_s + (wm * (BM / WM) + i * 32 + (lane & 31)) * RB + slot);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[j] = *reinterpret_cast<const vec_t<H, 8>*>(b_s + (wn * (BN / WN) + j * 32 + (lane & 31)) * RB + slot);
      if constexpr (AMODE == AM_SCALE) {
        const float* scs = reinterpret_cast<const float*>(b_s + B_BYTES) + s * 16 + (lane >> 5) * 8;
        const float4 s0 = ld4(scs), s1 = ld4(scs + 4);
        const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e) a[i][e] = (H)((float)a[i][e] * sv[e]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x16(a[i], b[j], acc[i][j]);
    }
  };

  // CM_LNBWD (16-bit C): the epilogue's x / dres chunks and row statistics loaded now, under the K loop.  Issued before
  // the ring's prologue DMAs: the first counted retire then also covers them, and they complete first.  64 x 256 tiles
  // (the 32 x 32 level's conv1 / conv4 dgrads): 22.3 -> 20.0 us per launch in the step trace; the same preload of the
  // residual chunk in the CM_PLAIN / CM_RESLN epilogues measured neutral in the step (1236 vs 1236 img/s) and was
  // not kept
  constexpr bool LPRE = CMODE == CM_LNBWD && sizeof(TC) == 2 && EPP == 1;
  constexpr int NPRE = LPRE ? (BM * (BN / 8) + 64 * NW - 1) / (64 * NW) : 0;
  LnPre<(NPRE > 0 ? NPRE : 1)> lpre;
  if constexpr (LPRE) {
#pragma unroll
    for (int it = 0; it < NPRE; ++it) {
      const int e = tid + it * 64 * NW, row = e / (BN / 8), c8 = (e % (BN / 8)) * 8;
      const int grow = m0 + row, gcol = n0 + c8;
      lpre.x[it] = lpre.r[it] = make_uint4(0, 0, 0, 0);
      lpre.st[it] = make_float2(0.f, 1.f);
      if (e < BM * (BN / 8) && grow < M && gcol < N) {
        const long off = (long)grow * N + gcol;
        lpre.x[it] = *reinterpret_cast<const uint4*>(reinterpret_cast<const TC*>(p.R) + off);
        lpre.r[it] = *reinterpret_cast<const uint4*>(reinterpret_cast<const TC*>(p.dres) + off);
        lpre.st[it] = p.stats_in[grow];
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NS - 1; ++t)
    if (t < nk) issue(t);
  GEMM_STAMP(2);
  for (int t = 0; t < nk; ++t) {
    // retire K-tile t (this wave's DMAs), leaving the later tiles of the ring in flight; the barrier then makes every
    // wave's part of tile t visible and frees the stage read at step t - 1 for tile t + NS - 1
    if (NS >= 5 && t + 3 < nk) wait_vm<3 * G>();
    else if (NS >= 4 && t + 2 < nk) wait_vm<2 * G>();
    else if (NS >= 3 && t + 1 < nk) wait_vm<G>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t == 0) GEMM_STAMP(3);
    if (t + NS - 1 < nk) issue(t + NS - 1);
    compute(t % NS);
  }
  GEMM_STAMP(4);
  __syncthreads();  // the ring is drained (vmcnt(0) at the last step); every fragment read done before Cs aliases it
  gemm_epilogue<BM, BN, CMODE, TC, H, WN, WM, EPP, NPRE>(p, acc, smem, m0, n0, &lpre);
#ifdef NBP_GEMM_PROBE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores landed
  GEMM_STAMP(5);
#endif
}

// ---------------------------------------------------------------- skinny GEMM (N, K <= 64), bf16 in / out
// The transposed product C^T = W . A^T on 32x32x16 MFMA: the weight is the A-operand (kept in registers for the whole
// launch: N, K <= 64), the pixel rows are the B-operand, loaded straight from global memory in fragment order (lane l
// reads 16 bytes of row l & 31 — no LDS, no barriers).  Each wave streams 32-pixel tiles, prefetching the next tile's
// fragments while the current one is multiplied; a lane ends up owning one pixel's channels (4 consecutive per
// register group), so the epilogue (bias, layer-scale residual, SimpleGate forward / backward) runs in registers and
// stores 8 / 16-byte pieces that complete whole rows in L2.
// The weight-gradient folds' LDS tiles (row-per-lane 16-byte stores, ds_read_b64_tr_b16 reads of 4 consecutive rows):
// the 16-byte chunk index of a row XOR-swizzled by (row / 4) mod 4.  With 64-byte rows the plain layout puts the 16
// lanes of a store on 4 chunk slots (4-way conflicts; 8-way for the 4-byte gate stores) -- measured 58 % of the
// conv5-fold kernel's LDS-active cycles as bank conflicts; the 4 rows of a transposed read share row / 4, so they keep
// one conflict-free 256-byte pattern.  (Not in the conv1 fold: at its 256 VGPRs even the one-XOR-per-side form spills
// 2 in the fp16 build, measured -0.3 % against its 32 % conflicted LDS cycles; profiles/r05_swz1/.)
__device__ __forceinline__ int fswz(int row, int col) {
  return (col & ~31) | ((((col >> 3) ^ (row >> 2)) & 3) << 3) | (col & 7);
}

template <typename H>
struct SkinnyP {
  const H* A;
  long lda;
  const float* a_scale;
  int rows_per_img;
  const H* W;
  long ldw;
  H* C;
  long ldc;
  int M, N, K;
  const float* bias;
  const H* R;
  const float* rscale;
  H* aux;
  // CM_LNBWD (LayerNorm2d backward in the epilogue, arch_util.py:277-289): the GEMM output is dn; R = the LN input x,
  // stats = (mu, sqrt(var + eps)) per row, lnw = the LN weight, dres = the residual-branch gradient added to dx;
  // per-block partials of sum(dn * yhat) / sum(dn) go to slab_w / slab_b [grid][N]
  const float2* stats;
  const float* lnw;
  const H* dres;
  float* slab_w;
  float* slab_b;
  // CM_RESLN (bias + layer-scale residual, then the next LayerNorm2d forward, arch_util.py:266-275): C = the stored
  // residual sum, nout = LN(C) with lnw / lnb_f, stats_out = (mu, sqrt(var + eps)) per row
  const float* lnb_f;
  H* nout;
  float2* stats_out;
  float eps;
  // CM_SGBWD_RC (SimpleGate backward with the gate input recomputed): t = A2 W2^T + b2 (the conv4 forward, its
  // output rows interleaved as stored, 2N columns) is rebuilt per tile on MFMA instead of being read from memory
  const H* A2;
  const H* W2;
  const float* b2;
  // WGF (with CM_SGBWD_RC at N = K = 32): the weight gradients that read this kernel's operands, per-block partials
  // U = dout^T g (g = the SimpleGate output rebuilt from t), V = colsum dout, dW2 = C^T A2 (C = the stored dt), db2 =
  // colsum C into slab_u [grid][N N], slab_v [grid][N], slab_w2 [grid][2N K], slab_b2 [grid][2N]
  float* slab_u;
  float* slab_v;
  float* slab_w2;
  float* slab_b2;
};

// CM_FFN (the level-0 NAFBlock FFN half, NAFNet_arch.py:74-80, N = K = 32): conv4 -> SimpleGate -> conv5 in one pass.
// The conv4 weight / bias are held like CM_SGBWD_RC's (W2 / b2: 2N interleaved rows), A = n2; t = A W2^T + b2 is
// formed on MFMA per 32-row tile exactly as the CM_SG kernel forms it, the gate g = t[2c] t[2c+1] (an fp32 product
// rounded once to H, as CM_SG stores it) never leaves the registers: the two lanes of a pixel (l, l ^ 32) swap half of
// their gates so each holds the 8 consecutive channels of a B-operand fragment, and conv5 (W = its weight) runs on
// them.  The epilogue is CM_RESLN's (bias, layer-scale residual R + rscale v, the next LayerNorm when nout is given).
// g2 (written and re-read by the two-launch form) is never stored: the level-0 backward rebuilds it from n2.
template <int NT, int KS, int AMODE, int CMODE, typename H, bool WGF = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WGF ? 2 : 1)))
void gemm_skinny_kernel(SkinnyP<H> p) {
  constexpr int LDT = NT * 32 + 4;  // fp32 row stride of the wave's staging tile
  constexpr bool FFN = CMODE == CM_FFN;
  static_assert(!FFN || (NT == 1 && KS == 2), "FFN fusion: the level-0 block (N = K = 32)");
  constexpr bool RESLN = CMODE == CM_RESLN || FFN;
  constexpr bool RC = CMODE == CM_SGBWD_RC;
  constexpr bool WGR = WGF && RC;                 // conv5's U / V + conv4's dW / db (nbp_dgrad_sg_rc_wg)
  constexpr bool WG1 = WGF && CMODE == CM_LNBWD;  // conv1's dW / db (nbp_dgrad_ln_bwd_wg)
  static_assert(!WGF || (WGR && NT == 1 && KS == 2) || (WG1 && NT == 1 && KS == 4),
                "weight-gradient folds: level-0 conv5 dgrad (N = K = 32), level-0 conv1 dgrad (N = 32, K = 64)");
  // bf16 row stride of the recomputed gate-input tile (RC) / of the rebuilt n1 tile (WG1)
  constexpr int LDT2 = RC ? 2 * NT * 32 + 8 : (WG1 ? 32 : 8);
  __shared__ float stage[4][32 * LDT];
  __shared__ __attribute__((aligned(16))) H stage2[4][32 * LDT2];
  // WGF: the tile's dt (32 rows x 64, 192-byte rows: conflict-free ds_read_b64_tr_b16), later the block's reduction
  __shared__ __attribute__((aligned(16))) H stage3[WGF ? 4 : 1][WGF ? 32 * 96 : 8];
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  float* tileS = stage[threadIdx.x >> 6];
  H* tileT = stage2[threadIdx.x >> 6];
  const int M = p.M, N = p.N, K = p.K;
  // RC / FFN: the conv4 weight (2N rows, K = the conv4 input width = this GEMM's K) and bias in registers
  constexpr int NT2 = RC || FFN ? 2 * NT : 1;
  vec_t<H, 8> w2[NT2][KS];
  float b2r[NT2][4][4];
  if constexpr (RC || FFN) {
#pragma unroll
    for (int t = 0; t < NT2; ++t) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int n = t * 32 + r, k = ks * 16 + 8 * h;
        vec_t<H, 8> v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
        if (n < 2 * N && k < K) v = *reinterpret_cast<const vec_t<H, 8>*>(p.W2 + (long)n * K + k);
        w2[t][ks] = v;
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = t * 32 + 8 * g + 4 * h + q;
          b2r[t][g][q] = c < 2 * N ? p.b2[c] : 0.f;
        }
    }
  }
  vec_t<H, 8> w[NT][KS];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int n = t * 32 + r, k = ks * 16 + 8 * h;
      vec_t<H, 8> v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
      if (n < N && k < K) v = *reinterpret_cast<const vec_t<H, 8>*>(p.W + (long)n * p.ldw + k);
      w[t][ks] = v;
    }
  // coalesced epilogue geometry: chunks of 8 output elements, row-major over the 32-row tile.  The output row holds
  // N elements (2N for the SimpleGate backward), so a lane's chunk column is fixed across its chunks.
  const int outw = (CMODE == CM_SGBWD || RC ? 2 : 1) * N;
  const int cpr = outw / 8;                                    // chunks per row (divides 64: outw in {8..128})
  const int ccol = (lane % cpr) * 8;                           // this lane's output column
  const int rstep = 64 / cpr;                                  // rows advanced per pass
  float bia[8], rsc[8], aw[8], ab[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bia[j] = 0.f; rsc[j] = 1.f; aw[j] = ab[j] = 0.f; }
  // WGF accumulators: dW2 (2 x 32 rows of dt channels x 32 n2 channels), U (32 x 32), V (this lane's 16 dout channels)
  floatx16 accw[2], accu;
  float vsum[KS][8];
#pragma unroll
  for (int i = 0; i < 16; ++i) accw[0][i] = accw[1][i] = accu[i] = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e) vsum[ks][e] = 0.f;
  if (RESLN && p.nout) {  // aw / ab hold the LN weight / bias of this lane's 8 columns
    const float4 w0 = ld4(p.lnw + ccol), w1 = ld4(p.lnw + ccol + 4), b0 = ld4(p.lnb_f + ccol), b1 = ld4(p.lnb_f + ccol + 4);
    aw[0] = w0.x; aw[1] = w0.y; aw[2] = w0.z; aw[3] = w0.w; aw[4] = w1.x; aw[5] = w1.y; aw[6] = w1.z; aw[7] = w1.w;
    ab[0] = b0.x; ab[1] = b0.y; ab[2] = b0.z; ab[3] = b0.w; ab[4] = b1.x; ab[5] = b1.y; ab[6] = b1.z; ab[7] = b1.w;
  }
  if (CMODE == CM_LNBWD) {  // rsc holds the LN weight of this lane's 8 columns
    const float4 s0 = ld4(p.lnw + ccol), s1 = ld4(p.lnw + ccol + 4);
    rsc[0] = s0.x; rsc[1] = s0.y; rsc[2] = s0.z; rsc[3] = s0.w; rsc[4] = s1.x; rsc[5] = s1.y; rsc[6] = s1.z; rsc[7] = s1.w;
    if (WG1) {  // bia holds the LN bias (n1 = lnw yhat + lnb rebuilt for the conv1 weight gradient)
      const float4 b0 = ld4(p.lnb_f + ccol), b1 = ld4(p.lnb_f + ccol + 4);
      bia[0] = b0.x; bia[1] = b0.y; bia[2] = b0.z; bia[3] = b0.w; bia[4] = b1.x; bia[5] = b1.y; bia[6] = b1.z; bia[7] = b1.w;
    }
  } else if (CMODE != CM_SGBWD && !RC) {
    if (p.bias) {
      const float4 b0 = ld4(p.bias + ccol), b1 = ld4(p.bias + ccol + 4);
      bia[0] = b0.x; bia[1] = b0.y; bia[2] = b0.z; bia[3] = b0.w; bia[4] = b1.x; bia[5] = b1.y; bia[6] = b1.z; bia[7] = b1.w;
    }
    if (p.rscale) {
      const float4 s0 = ld4(p.rscale + ccol), s1 = ld4(p.rscale + ccol + 4);
      rsc[0] = s0.x; rsc[1] = s0.y; rsc[2] = s0.z; rsc[3] = s0.w; rsc[4] = s1.x; rsc[5] = s1.y; rsc[6] = s1.z; rsc[7] = s1.w;
    }
  }
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6), nwaves = (long)gridDim.x * 4;
  const long ntiles = (M + 31) / 32;
  auto load_a = [&](long tile, vec_t<H, 8>* a) {
    const long m = tile * 32 + r;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = ks * 16 + 8 * h;
      vec_t<H, 8> v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
      if (m < M && k < K) {
        v = *reinterpret_cast<const vec_t<H, 8>*>(p.A + m * p.lda + k);
        if (AMODE == AM_SCALE) {
          const float* sc = p.a_scale + (m / p.rows_per_img) * K + k;
          const float4 s0 = ld4(sc), s1 = ld4(sc + 4);
          const float f[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (H)((float)v[j] * f[j]);
        }
      }
      a[ks] = v;
    }
  };
  auto load_a2 = [&](long tile, vec_t<H, 8>* a) {  // RC: the conv4 input rows (plain, row stride K)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const long m = tile * 32 + r;
      const int k = ks * 16 + 8 * h;
      vec_t<H, 8> v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (H)0.f;
      if (m < M && k < K) v = *reinterpret_cast<const vec_t<H, 8>*>(p.A2 + m * K + k);
      a[ks] = v;
    }
  };
  vec_t<H, 8> a0[KS], a1[KS], c0[RC ? KS : 1], c1[RC ? KS : 1];
  long tile = wave;
  if (tile < ntiles) {
    load_a(tile, a0);
    if constexpr (RC) load_a2(tile, c0);
  }
  // CM_LNBWD: a row's cpr = 4 NT lanes are consecutive (N = 32 NT), so a lane's epilogue rows are lane / cpr + q * rstep
  // for q < 2 NT; their x / dres chunks and LN statistics are loaded before the tile's MFMAs (the latency then overlaps
  // the MFMAs and the LDS staging instead of following them)
  // (NT = 1 only: at NT = 2 the 4 preloaded rows cost more registers than the overlap gains -- measured 40 -> 50 us at
  // level 1, 69 -> 60 us at level 0; the same preload of the residual rows in the level-0 CM_RESLN epilogue measured
  // 61 -> 79 us, not kept)
  constexpr bool PRE = CMODE == CM_LNBWD && NT == 1;
  constexpr int NPL = PRE ? 2 * NT : 1;
  for (; tile < ntiles; tile += nwaves) {
    if (tile + nwaves < ntiles) {
      load_a(tile + nwaves, a1);
      if constexpr (RC) load_a2(tile + nwaves, c1);
    }
    vec_t<H, 8> xpre[NPL], rpre[NPL];
    float2 spre[NPL];
    if constexpr (PRE) {
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        const long m = tile * 32 + lane / cpr + q * rstep;
        if (m < M) {
          const long off = m * p.ldc + ccol;
          xpre[q] = *reinterpret_cast<const vec_t<H, 8>*>(p.R + off);
          rpre[q] = *reinterpret_cast<const vec_t<H, 8>*>(p.dres + off);
          spre[q] = p.stats[m];
        }
      }
    }
    floatx16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    if constexpr (FFN) {
      // conv4: lane (r, h) gets pixel r's t channels 32 t2 + 8 g + 4 h + q (rows interleaved), i.e. the gates
      // c = 16 t2 + 4 g + 2 h + {0, 1}
      vec_t<H, 2> gp[NT2][4];
#pragma unroll
      for (int t2 = 0; t2 < NT2; ++t2) {
        floatx16 a2c;
#pragma unroll
        for (int i = 0; i < 16; ++i) a2c[i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a2c = mfma32x32x16(w2[t2][ks], a0[ks], a2c);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float pr0 = (a2c[4 * g] + b2r[t2][g][0]) * (a2c[4 * g + 1] + b2r[t2][g][1]);
          float pr1 = (a2c[4 * g + 2] + b2r[t2][g][2]) * (a2c[4 * g + 3] + b2r[t2][g][3]);
          asm volatile("" : "+v"(pr0), "+v"(pr1));  // an fp32 product, then one rounding (no fused mix-precision op)
          gp[t2][g][0] = (H)pr0;
          gp[t2][g][1] = (H)pr1;
        }
      }
      // conv5's B fragment of K step ks = t2: lane h needs gates 16 t2 + 8 h + [0, 8); it holds g = 2h, 2h + 1 of
      // them and its partner (lane ^ 32) the other two
#pragma unroll
      for (int t2 = 0; t2 < NT2; ++t2) {
        const vec_t<H, 2> s0 = h ? gp[t2][0] : gp[t2][2], s1 = h ? gp[t2][1] : gp[t2][3];
        const vec_t<H, 2> r0 = __builtin_bit_cast(vec_t<H, 2>, __shfl_xor(__builtin_bit_cast(int, s0), 32, 64));
        const vec_t<H, 2> r1 = __builtin_bit_cast(vec_t<H, 2>, __shfl_xor(__builtin_bit_cast(int, s1), 32, 64));
        const vec_t<H, 2> q0 = h ? r0 : gp[t2][0], q1 = h ? gp[t2][2] : r0;
        const vec_t<H, 2> q2 = h ? r1 : gp[t2][1], q3 = h ? gp[t2][3] : r1;
        vec_t<H, 8> bg;
        bg[0] = q0[0]; bg[1] = q0[1]; bg[2] = q1[0]; bg[3] = q1[1];
        bg[4] = q2[0]; bg[5] = q2[1]; bg[6] = q3[0]; bg[7] = q3[1];
        acc[0] = mfma32x32x16(w[0][t2], bg, acc[0]);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma32x32x16(w[t][ks], a0[ks], acc[t]);
    }
    // lane (r, h) owns pixel r, channels t*32 + 8g + 4h + {0..3}: stage as rows of the tile
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(tileS + r * LDT + t * 32 + 8 * g + 4 * h) =
            make_float4(acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]);
    // WGF: the SimpleGate outputs g = (t[2c] t[2c+1]) of this lane's channels, from the fp32 t exactly as the conv4
    // forward's SimpleGate epilogue computed them (its stored g)
    vec_t<H, 2> g2h[NT2][4];
    if constexpr (RC) {  // t = bf16(A2 W2^T + b2) exactly as the conv4 forward stored it (same MFMA sequence)
#pragma unroll
      for (int t = 0; t < NT2; ++t) {
        floatx16 a2c;
#pragma unroll
        for (int i = 0; i < 16; ++i) a2c[i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) a2c = mfma32x32x16(w2[t][ks], c0[ks], a2c);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          vec_t<H, 4> o;
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[q] = a2c[4 * g + q] + b2r[t][g][q];
            o[q] = (H)v[q];
          }
          *reinterpret_cast<vec_t<H, 4>*>(tileT + r * LDT2 + t * 32 + 8 * g + 4 * h) = o;
          if constexpr (WGF) {
            float pr0 = v[0] * v[1], pr1 = v[2] * v[3];
            asm volatile("" : "+v"(pr0), "+v"(pr1));  // the forward's gate: an fp32 product, then one rounding
            g2h[t][g][0] = (H)pr0;
            g2h[t][g][1] = (H)pr1;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    const long m0 = tile * 32;
    if constexpr (PRE) {  // dx = (g - yhat mean(g yhat) - mean(g)) / den + dres, g = dn * lnw
      constexpr int G = 4 * NT;
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        const int rr = lane / cpr + q * rstep;
        const long m = m0 + rr;
        if (m >= M) {
          if constexpr (WG1) {  // the fold's n1 tile: zero rows past M (their dt1 rows are zero, stale data could be NaN)
            vec_t<H, 8> z;
#pragma unroll
            for (int j = 0; j < 8; ++j) z[j] = (H)0.f;
            *reinterpret_cast<vec_t<H, 8>*>(tileT + rr * LDT2 + ccol) = z;
            continue;
          }
          break;
        }
        const float4 u0 = *reinterpret_cast<const float4*>(tileS + rr * LDT + ccol);
        const float4 u1 = *reinterpret_cast<const float4*>(tileS + rr * LDT + ccol + 4);
        const float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
        const float2 st = spre[q];
        const float inv = 1.f / st.y;
        float yh[8], sg = 0.f, sgy = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          yh[j] = ((float)xpre[q][j] - st.x) * inv;
          const float g = v[j] * rsc[j];
          sg += g;
          sgy = fmaf(g, yh[j], sgy);
          aw[j] = fmaf(v[j], yh[j], aw[j]);
          ab[j] += v[j];
        }
        if constexpr (WG1) {  // n1 exactly as the forward LayerNorm stored it (nbp_ln_fwd_nhwc / the RESLN epilogue)
          vec_t<H, 8> nn;
#pragma unroll
          for (int j = 0; j < 8; ++j) nn[j] = (H)fmaf(rsc[j], yh[j], bia[j]);
          *reinterpret_cast<vec_t<H, 8>*>(tileT + rr * LDT2 + ccol) = nn;
        }
        sg = group_sum<G>(sg);
        sgy = group_sum<G>(sgy);
        const float mg = sg / (float)N, mgy = sgy / (float)N;
        vec_t<H, 8> o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (H)((v[j] * rsc[j] - yh[j] * mgy - mg) * inv + (float)rpre[q][j]);
        *reinterpret_cast<vec_t<H, 8>*>(p.C + m * p.ldc + ccol) = o;
      }
    }
    for (int rr = lane / cpr; !PRE && rr < 32; rr += rstep) {
      const long m = m0 + rr;
      if (m >= M) {
        if constexpr (WGR) {  // the fold's dt tile: zero rows past M (their n2 rows are zero, stale data could be NaN)
          vec_t<H, 8> z;
#pragma unroll
          for (int j = 0; j < 8; ++j) z[j] = (H)0.f;
          *reinterpret_cast<vec_t<H, 8>*>(stage3[threadIdx.x >> 6] + rr * 96 + ccol) = z;
          continue;
        }
        break;
      }
      if (CMODE == CM_SGBWD || RC) {  // chunk = 4 gates (interleaved pairs): dg from the tile, t from R (or rebuilt)
        const float4 dg = *reinterpret_cast<const float4*>(tileS + rr * LDT + ccol / 2);
        const long off = m * p.ldc + ccol;
        const vec_t<H, 8> tv = RC ? *reinterpret_cast<const vec_t<H, 8>*>(tileT + rr * LDT2 + ccol)
                             : *reinterpret_cast<const vec_t<H, 8>*>(p.R + off);
        const float d[4] = {dg.x, dg.y, dg.z, dg.w};
        vec_t<H, 8> o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[2 * j] = (H)(d[j] * (float)tv[2 * j + 1]);
          o[2 * j + 1] = (H)(d[j] * (float)tv[2 * j]);
        }
        *reinterpret_cast<vec_t<H, 8>*>(p.C + off) = o;
        if constexpr (WGR) {
          *reinterpret_cast<vec_t<H, 8>*>(stage3[threadIdx.x >> 6] + rr * 96 + ccol) = o;
#pragma unroll
          for (int j = 0; j < 8; ++j) ab[j] += (float)o[j];  // db2 partial of this lane's 8 columns
        }
        continue;
      }
      const float4 u0 = *reinterpret_cast<const float4*>(tileS + rr * LDT + ccol);
      const float4 u1 = *reinterpret_cast<const float4*>(tileS + rr * LDT + ccol + 4);
      float v[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      if constexpr (CMODE == CM_LNBWD) {  // (NT > 1) the row's cpr lanes are consecutive: shuffle sums in the group
        constexpr int G = 4 * NT;
        const long off = m * p.ldc + ccol;
        const vec_t<H, 8> xv = *reinterpret_cast<const vec_t<H, 8>*>(p.R + off);
        const vec_t<H, 8> rv = *reinterpret_cast<const vec_t<H, 8>*>(p.dres + off);
        const float2 st = p.stats[m];
        const float inv = 1.f / st.y;
        float yh[8], sg = 0.f, sgy = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          yh[j] = ((float)xv[j] - st.x) * inv;
          const float g = v[j] * rsc[j];
          sg += g;
          sgy = fmaf(g, yh[j], sgy);
          aw[j] = fmaf(v[j], yh[j], aw[j]);
          ab[j] += v[j];
        }
        sg = group_sum<G>(sg);
        sgy = group_sum<G>(sgy);
        const float mg = sg / (float)N, mgy = sgy / (float)N;
        vec_t<H, 8> o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (H)((v[j] * rsc[j] - yh[j] * mgy - mg) * inv + (float)rv[j]);
        *reinterpret_cast<vec_t<H, 8>*>(p.C + off) = o;
        continue;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bia[j];
      const long off = m * p.ldc + ccol;
      if ((CMODE == CM_PLAIN || RESLN) && p.R) {
        const vec_t<H, 8> rv = *reinterpret_cast<const vec_t<H, 8>*>(p.R + off);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (float)rv[j] + rsc[j] * v[j];
      }
      vec_t<H, 8> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (H)v[j];
      if (CMODE != CM_SG || p.C) *reinterpret_cast<vec_t<H, 8>*>(p.C + off) = o;  // SG: t may be dropped (recomputed)
      if (RESLN && p.nout) {  // LayerNorm2d of the stored (bf16) row, as ln_fwd_nhwc computes it
        constexpr int G = 4 * NT;
        float xv[8], sm = 0.f, q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[j] = (float)o[j];
          sm += xv[j];
        }
        sm = group_sum<G>(sm);
        const float mu = sm / (float)N;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = xv[j] - mu;
          q = fmaf(d, d, q);
        }
        q = group_sum<G>(q);
        const float dd = sqrtf(q / (float)N + p.eps), inv = 1.f / dd;
        vec_t<H, 8> nn;
#pragma unroll
        for (int j = 0; j < 8; ++j) nn[j] = (H)fmaf(aw[j], (xv[j] - mu) * inv, ab[j]);
        *reinterpret_cast<vec_t<H, 8>*>(p.nout + m * N + ccol) = nn;
        if (ccol == 0) p.stats_out[m] = make_float2(mu, dd);
      }
      if (CMODE == CM_SG) {  // g[c] = t[2c] * t[2c+1]: 4 gates of this chunk
        vec_t<H, 4> gv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float pr = v[2 * j] * v[2 * j + 1];
          asm volatile("" : "+v"(pr));  // an fp32 product, then one rounding (as CM_FFN forms the gate)
          gv[j] = (H)pr;
        }
        *reinterpret_cast<vec_t<H, 4>*>(p.aux + m * (p.ldc / 2) + ccol / 2) = gv;
      }
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (WG1) {
      // stage dt1 (this GEMM's A) next to the rebuilt n1 tile, then accumulate dW1 += dt1^T n1 over the tile's 32 rows
      // with transposed fragment reads (WGR's dW2 pattern; rows past M are zero in both tiles)
      H* st = stage3[threadIdx.x >> 6];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        *reinterpret_cast<vec_t<H, 8>*>(st + r * 96 + ks * 16 + 8 * h) = a0[ks];
#pragma unroll
        for (int e = 0; e < 8; ++e) vsum[ks][e] += (float)a0[ks][e];  // db1 partial
      }
      __builtin_amdgcn_wave_barrier();
      const int grp = lane >> 4, gq = (lane & 15) >> 2, pp = lane & 3;
      const int fcol = 16 * (grp & 1) + 4 * pp;
#pragma unroll
      for (int ks = 0; ks < 32; ks += 16) {
        vec_t<H, 8> fa[2], fn;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int row = ks + 8 * h + 4 * tt + gq;
          const vec_t<H, 4> a0v = ds_read_tr16<H>(st + row * 96 + fcol);
          const vec_t<H, 4> a1v = ds_read_tr16<H>(st + row * 96 + 32 + fcol);
          const vec_t<H, 4> nv = ds_read_tr16<H>(tileT + row * LDT2 + fcol);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            fa[0][4 * tt + e] = a0v[e];
            fa[1][4 * tt + e] = a1v[e];
            fn[4 * tt + e] = nv[e];
          }
        }
        accw[0] = mfma32x32x16(fa[0], fn, accw[0]);
        accw[1] = mfma32x32x16(fa[1], fn, accw[1]);
      }
      __builtin_amdgcn_wave_barrier();
    }
    if constexpr (WGR) {
      // stage dout (this GEMM's A) and n2 (A2) in the dead fp32 tile, g in the dead t tile (32-element rows), then
      // accumulate U += dout^T g and dW2 += dt^T n2 over the tile's 32 rows with transposed fragment reads
      H* sd = reinterpret_cast<H*>(tileS);
      H* sn = sd + 32 * 32;
      H* sg = tileT;
      const H* st = stage3[threadIdx.x >> 6];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        *reinterpret_cast<vec_t<H, 8>*>(sd + r * 32 + fswz(r, ks * 16 + 8 * h)) = a0[ks];
        *reinterpret_cast<vec_t<H, 8>*>(sn + r * 32 + fswz(r, ks * 16 + 8 * h)) = c0[ks];
#pragma unroll
        for (int e = 0; e < 8; ++e) vsum[ks][e] += (float)a0[ks][e];  // V partial (rows past M are zero-filled)
      }
#pragma unroll
      for (int t = 0; t < NT2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<vec_t<H, 2>*>(sg + r * 32 + fswz(r, t * 16 + 4 * g + 2 * h)) = g2h[t][g];
      __builtin_amdgcn_wave_barrier();
      const int grp = lane >> 4, gq = (lane & 15) >> 2, pp = lane & 3;
      const int fcol = 16 * (grp & 1) + 4 * pp;
#pragma unroll
      for (int ks = 0; ks < 32; ks += 16) {
        vec_t<H, 8> fa[2], fn, fu, fg;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int row = ks + 8 * h + 4 * tt + gq;
          const vec_t<H, 4> a0v = ds_read_tr16<H>(st + row * 96 + fcol);
          const vec_t<H, 4> a1v = ds_read_tr16<H>(st + row * 96 + 32 + fcol);
          const vec_t<H, 4> nv = ds_read_tr16<H>(sn + row * 32 + fswz(row, fcol));
          const vec_t<H, 4> uv = ds_read_tr16<H>(sd + row * 32 + fswz(row, fcol));
          const vec_t<H, 4> gv = ds_read_tr16<H>(sg + row * 32 + fswz(row, fcol));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            fa[0][4 * tt + e] = a0v[e];
            fa[1][4 * tt + e] = a1v[e];
            fn[4 * tt + e] = nv[e];
            fu[4 * tt + e] = uv[e];
            fg[4 * tt + e] = gv[e];
          }
        }
        accw[0] = mfma32x32x16(fa[0], fn, accw[0]);
        accw[1] = mfma32x32x16(fa[1], fn, accw[1]);
        accu = mfma32x32x16(fu, fg, accu);
      }
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) a0[ks] = a1[ks];
    if constexpr (RC)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) c0[ks] = c1[ks];
  }
  if constexpr (WG1) {
    // block partials, waves combined in fixed order through stage3 (as fp32): [0, 2048) dW1 (row n = dt1 column,
    // col k = n1 channel), [2048, 2112) db1
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) vsum[ks][e] += __shfl_xor(vsum[ks][e], o, 64);  // lanes sharing h
    float* red = reinterpret_cast<float*>(&stage3[0][0]);
    const int wv = threadIdx.x >> 6;
    for (int w = 0; w < 4; ++w) {
      __syncthreads();
      if (wv == w) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int rr = 0; rr < 16; ++rr) {
            const int n = i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h, k = r;
            float* d = red + n * 32 + k;
            *d = (w == 0 ? 0.f : *d) + accw[i][rr];
          }
        if (r == 0)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float* d = red + 2048 + ks * 16 + 8 * h + e;
              *d = (w == 0 ? 0.f : *d) + vsum[ks][e];
            }
      }
    }
    __syncthreads();
    const long bb = blockIdx.x;
    for (int i = threadIdx.x; i < 2112; i += blockDim.x) {
      const float v = red[i];
      if (i < 2048) p.slab_w2[bb * 2048 + i] = v;
      else p.slab_b2[bb * 64 + i - 2048] = v;
    }
  }
  if constexpr (WGR) {
    // block partials, waves combined in fixed order through stage3 (as fp32): [0, 2048) dW2 (row n = dt column, col k =
    // n2 channel), [2048, 3072) U, [3072, 3136) db2, [3136, 3168) V
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int o = cpr; o < 64; o <<= 1) ab[j] += __shfl_xor(ab[j], o, 64);  // lanes sharing ccol
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) vsum[ks][e] += __shfl_xor(vsum[ks][e], o, 64);  // lanes sharing h
    float* red = reinterpret_cast<float*>(&stage3[0][0]);
    const int wv = threadIdx.x >> 6;
    for (int w = 0; w < 4; ++w) {
      __syncthreads();
      if (wv == w) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int rr = 0; rr < 16; ++rr) {
            const int n = i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h, k = r;
            float* d = red + n * 32 + k;
            *d = (w == 0 ? 0.f : *d) + accw[i][rr];
          }
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int n = (rr & 3) + 8 * (rr >> 2) + 4 * h, k = r;
          float* d = red + 2048 + n * 32 + k;
          *d = (w == 0 ? 0.f : *d) + accu[rr];
        }
        if (lane < cpr)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float* d = red + 3072 + ccol + j;
            *d = (w == 0 ? 0.f : *d) + ab[j];
          }
        if (r == 0)
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              float* d = red + 3136 + ks * 16 + 8 * h + e;
              *d = (w == 0 ? 0.f : *d) + vsum[ks][e];
            }
      }
    }
    __syncthreads();
    const long bb = blockIdx.x;
    for (int i = threadIdx.x; i < 3168; i += blockDim.x) {
      const float v = red[i];
      if (i < 2048) p.slab_w2[bb * 2048 + i] = v;
      else if (i < 3072) p.slab_u[bb * 1024 + i - 2048] = v;
      else if (i < 3136) p.slab_b2[bb * 64 + i - 3072] = v;
      else p.slab_v[bb * 32 + i - 3136] = v;
    }
  }
  if constexpr (CMODE == CM_LNBWD) {  // LN weight / bias gradient partials: lanes sharing ccol, then the 4 waves
    constexpr int G = 4 * NT;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int o = G; o < 64; o <<= 1) {
        aw[j] += __shfl_xor(aw[j], o, 64);
        ab[j] += __shfl_xor(ab[j], o, 64);
      }
    __syncthreads();
    float* red = &stage[0][0];  // [4 waves][2][N]
    const int wv = threadIdx.x >> 6;
    if (lane < G) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(wv * 2 + 0) * N + ccol + j] = aw[j];
        red[(wv * 2 + 1) * N + ccol + j] = ab[j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < N; c += blockDim.x) {
      p.slab_w[(long)blockIdx.x * N + c] = ((red[0 * N + c] + red[2 * N + c]) + red[4 * N + c]) + red[6 * N + c];
      p.slab_b[(long)blockIdx.x * N + c] = ((red[1 * N + c] + red[3 * N + c]) + red[5 * N + c]) + red[7 * N + c];
    }
  }
}

long skinny_blocks(long M) {
  const long ntiles = (M + 31) / 32;
  const long blocks = (ntiles + 3) / 4;
  // 4 blocks (16 waves) resident per CU: one round over the 256 CUs (768 / 1536 / 2048 measured within +-0.5 %)
  constexpr long cap = 1024;
  return blocks > cap ? cap : blocks;
}

// the weight-gradient fold kernels (WGF: 238-256 VGPRs, 2 waves per SIMD, so 2 blocks per CU resident): a grid of one
// resident round (512) instead of two -- each wave walks twice the tiles with its prefetch overlapped, and the fold
// slabs halve (A/B in the quick bench, fp16: 1350.2 / 1354.6 vs 1349.8 / 1347.8 img/s, eager level-0 backward 1.95 vs
// 2.02 ms; profiles/r05_wgcap/).  NBP_SKINNY_WG_CAP overrides (A/B only).
long skinny_wg_blocks(long M) {
  static const long cap = [] {
    const char* e = getenv("NBP_SKINNY_WG_CAP");
    return e ? atol(e) : 512L;
  }();
  const long b = skinny_blocks(M);
  return b > cap ? cap : b;
}

// NBP_SKINNY_OCC=0: every skinny kernel on skinny_blocks' grid (A/B)
bool skinny_occ_enabled() {
  static const bool on = [] {
    const char* e = getenv("NBP_SKINNY_OCC");
    return !e || atoi(e) != 0;
  }();
  return on;
}

// the grid of one skinny instantiation: its tiles in workgroups of 4 waves, at most one resident round (occupancy x
// CUs, from the HIP occupancy query: 2-4 workgroups per CU by its VGPRs) -- a second round re-pays the pipeline fill
// that the grid-stride tile loop otherwise overlaps (the fold kernels: +0.3 % with 512 instead of 1024)
template <int NT, int KS, int AMODE, int CMODE, typename H, bool WGF = false>
long skinny_grid(long M) {
  static const long cap = [] {
    int occ = 0, dev = 0, ncu = 0;
    if (!skinny_occ_enabled() || hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, gemm_skinny_kernel<NT, KS, AMODE, CMODE, H, WGF>, 256, 0) !=
            hipSuccess || occ <= 0 || ncu <= 0)
      return 1024L;
    return (long)occ * ncu;
  }();
  const long b = skinny_blocks(M);
  return b > cap ? cap : b;
}

// K <= 64 in 16-wide steps, or K <= 128 (KS = 8, the level-1 conv4 / conv1 dgrads); returns the grid (workgroups)
template <int AMODE, int CMODE, typename H>
long launch_skinny(const SkinnyP<H>& p, hipStream_t st) {
  long nb = 0;
  const int nt = (p.N + 31) / 32, ks = (p.K + 15) / 16;
#define NBP_SKINNY(NT_, KS_)                                          \
  (nb = skinny_grid<NT_, KS_, AMODE, CMODE, H>(p.M),                  \
   gemm_skinny_kernel<NT_, KS_, AMODE, CMODE, H><<<dim3((unsigned)nb), 256, 0, st>>>(p))
  if (nt == 1) {
    if (ks == 1) NBP_SKINNY(1, 1); else if (ks == 2) NBP_SKINNY(1, 2); else if (ks == 3) NBP_SKINNY(1, 3);
    else if (ks == 4) NBP_SKINNY(1, 4); else NBP_SKINNY(1, 8);
  } else {
    if (ks == 1) NBP_SKINNY(2, 1); else if (ks == 2) NBP_SKINNY(2, 2); else if (ks == 3) NBP_SKINNY(2, 3);
    else if (ks == 4) NBP_SKINNY(2, 4); else NBP_SKINNY(2, 8);
  }
#undef NBP_SKINNY
  return nb;
}

// whether the skinny path serves this call (bf16 in / out, N and K <= 64, supported modes, aligned rows)
template <typename H>
bool try_skinny(const void* A, long lda, int a_mode, const float* a_scale, int rows, const void* Bw, long ldb, void* C,
                long ldc, int c_mode, int M, int N, int K, const float* bias, const void* R, const float* rscale,
                void* pre, hipStream_t st) {
  if (N > 64 || K > 128 || N % 8 || K % 8 || lda % 8 || ldb % 8 || ldc % 8) return false;
  const bool ok = (a_mode == AM_PLAIN && c_mode == CM_PLAIN && !pre) || (a_mode == AM_SCALE && c_mode == CM_PLAIN && !pre) ||
                  (a_mode == AM_PLAIN && c_mode == CM_SG) || (a_mode == AM_SCALE && c_mode == CM_SGBWD) ||
                  (a_mode == AM_PLAIN && c_mode == CM_SGBWD);
  if (!ok) return false;
  SkinnyP<H> p{reinterpret_cast<const H*>(A), lda, a_scale, rows, reinterpret_cast<const H*>(Bw), ldb,
            reinterpret_cast<H*>(C), ldc, M, N, K, bias, reinterpret_cast<const H*>(R), rscale,
            reinterpret_cast<H*>(pre), nullptr, nullptr, nullptr, nullptr, nullptr};
  if (c_mode == CM_SG) launch_skinny<AM_PLAIN, CM_SG, H>(p, st);
  else if (c_mode == CM_SGBWD && a_mode == AM_SCALE) launch_skinny<AM_SCALE, CM_SGBWD, H>(p, st);
  else if (c_mode == CM_SGBWD) launch_skinny<AM_PLAIN, CM_SGBWD, H>(p, st);
  else if (a_mode == AM_SCALE) launch_skinny<AM_SCALE, CM_PLAIN, H>(p, st);
  else launch_skinny<AM_PLAIN, CM_PLAIN, H>(p, st);
  return true;
}

// fp32 flat parameters -> 16-bit copy (all; eight elements per thread, 16-byte stores), plus transposed 16-bit copies
// of the listed [rows][cols] matrices
template <typename H>
__global__ __launch_bounds__(256) void cvt_bf16_kernel(const float* __restrict__ src, long n, H* __restrict__ dst) {
  const long n8 = n / 8, stride = (long)gridDim.x * blockDim.x;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const float4 a = ld4(src + 8 * i), b = ld4(src + 8 * i + 4);
    vec_t<H, 8> v;
    v[0] = (H)a.x; v[1] = (H)a.y; v[2] = (H)a.z; v[3] = (H)a.w;
    v[4] = (H)b.x; v[5] = (H)b.y; v[6] = (H)b.z; v[7] = (H)b.w;
    *reinterpret_cast<vec_t<H, 8>*>(dst + 8 * i) = v;
  }
  for (long i = 8 * n8 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = (H)src[i];
}

// desc: [ndesc][4] int64 {offset, rows, cols, row-scale offset or -1}; block (x: tile index, y: matrix).  With a
// row scale s (the layer scale beta / gamma of conv3 / conv5) the copy is (diag(s) W)^T.  64 x 64 tiles: float4 row
// reads (cols a multiple of 4), transposed rows leave as 4-element (8-byte) stores (rows a multiple of 4).
template <typename H>
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const float* __restrict__ src, const long* __restrict__ desc,
                                                             H* __restrict__ dst_t) {
  __shared__ float tile[64][65];
  const long off = desc[blockIdx.y * 4], R = desc[blockIdx.y * 4 + 1], Cc = desc[blockIdx.y * 4 + 2];
  const long soff = desc[blockIdx.y * 4 + 3];
  const long tiles_c = (Cc + 63) / 64, ntiles = ((R + 63) / 64) * tiles_c;
  const int tid = threadIdx.x;
  const bool vec = (Cc & 3) == 0 && (R & 3) == 0 && (off & 3) == 0;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long r0 = (t / tiles_c) * 64, c0 = (t % tiles_c) * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rr = (tid >> 4) + 16 * k, cc = (tid & 15) * 4;
      const long r = r0 + rr, c = c0 + cc;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < R) {
        const float sc = soff >= 0 ? src[soff + r] : 1.f;
        if (vec && c + 3 < Cc) {
          const float4 q = ld4(src + off + r * Cc + c);
          v[0] = q.x * sc; v[1] = q.y * sc; v[2] = q.z * sc; v[3] = q.w * sc;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (c + j < Cc) v[j] = src[off + r * Cc + c + j] * sc;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) tile[rr][cc + j] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int q = tid + 256 * k, ci = q >> 4, rq = (q & 15) * 4;
      const long c = c0 + ci, r = r0 + rq;
      if (c >= Cc || r >= R) continue;
      H* d = dst_t + off + c * R + r;
      if (vec) {
        vec_t<H, 4> o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (H)tile[rq + j][ci];
        *reinterpret_cast<vec_t<H, 4>*>(d) = o;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (r + j < R) d[j] = (H)tile[rq + j][ci];
      }
    }
    __syncthreads();
  }
}

// NBP_GLDS=0 (read per launch): the register-staged tiles instead of the LDS-DMA ones -- the reference path of the
// bitwise tests (tests/test_gpu_glds.py: same tiles, fragment order and MFMA sequence).  Unset: LDS-DMA, the ring
// depth chosen per launch by glds_auto_depth.
int glds_depth() {
  const char* e = getenv("NBP_GLDS");
  return e && e[0] == '0' ? 0 : -1;
}

int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

// Auto ring depth: the deepest ring (<= 4, <= nmax) with which every CU still holds all the blocks the grid gives it
// (LDS per block = max(depth x stage, fp32 C staging)).  The small-grid deep-level GEMMs (2 blocks per CU, 8 K-steps,
// memory-latency bound) get 3 / 4 tiles in flight; large grids keep 2 and their blocks per CU.
int glds_auto_depth(long blocks, int stage_bytes, int c_bytes, int nmax) {
  const long per_cu = (blocks + cu_count() - 1) / cu_count();
  for (int d = nmax; d > 2; --d) {
    const long lds = (long)d * stage_bytes > c_bytes ? (long)d * stage_bytes : c_bytes;
    if (per_cu * lds <= 160L * 1024) return d;
  }
  return 2;
}


template <int BM, int BN, int AMODE, int CMODE, typename TA, typename TC, typename H>
void launch(const GemmPB& p, hipStream_t st) {
  dim3 grid(cdiv(p.M, BM), cdiv(p.N, BN));
  if constexpr (sizeof(TA) == 2 && (AMODE == AM_PLAIN || AMODE == AM_SCALE || AMODE == AM_S2D || AMODE == AM_IM2COL)) {
    const int ns_env = glds_depth();
    const int ns = ns_env < 0 ? 2 : ns_env;
    // 16-byte aligned sources (lda, ldb, cs multiples of 8); a tile's rows in one image for the per-image scale
    const bool ok = ns >= 2 && p.K > 32 && p.ldb % 8 == 0 &&
                    (AMODE == AM_S2D || AMODE == AM_IM2COL ? p.cs % 8 == 0 : p.lda % 8 == 0) &&
                    (AMODE != AM_SCALE || p.rows_per_img % BM == 0);
    if (ok) {
      // the ring depth the tile's LDS allows (stage = (BM + BN) x 128 B + scales; the fp32 C staging must fit too)
      constexpr int STB = (BM + BN) * 128 + (AMODE == AM_SCALE ? 256 : 0), CB = BM * (BN + 4) * 4;
#ifdef NBP_GEMM_NS5  // probe builds only: a 5-deep ring where it fits
      constexpr int NMAX = 5 * STB <= 160 * 1024 && CB <= 160 * 1024 ? 5 :
                           4 * STB <= 160 * 1024 && CB <= 160 * 1024 ? 4 : (3 * STB <= 160 * 1024 ? 3 : 2);
#else
      constexpr int NMAX = 4 * STB <= 160 * 1024 && CB <= 160 * 1024 ? 4 : (3 * STB <= 160 * 1024 ? 3 : 2);
#endif
      const int nd = ns_env < 0 ? glds_auto_depth((long)grid.x * grid.y, STB, CB, NMAX) : (ns < NMAX ? ns : NMAX);
      if constexpr (BN >= 128 && CMODE != CM_LNBWD && CMODE != CM_CHANDOT) {
        // 2 x 4 waves of (BM / 2) x (BN / 4), two per SIMD (+2 % step over 2 x 2 waves)
        if (nd == 2) gemm_glds_kernel<BM, BN, 2, AMODE, CMODE, TC, H, 4><<<grid, 512, 0, st>>>(p);
        else if (nd == 3) gemm_glds_kernel<BM, BN, (NMAX >= 3 ? 3 : 2), AMODE, CMODE, TC, H, 4><<<grid, 512, 0, st>>>(p);
        else if (nd == 4 || NMAX < 5) gemm_glds_kernel<BM, BN, (NMAX >= 4 ? 4 : 2), AMODE, CMODE, TC, H, 4><<<grid, 512, 0, st>>>(p);
        else gemm_glds_kernel<BM, BN, (NMAX >= 5 ? 5 : 2), AMODE, CMODE, TC, H, 4><<<grid, 512, 0, st>>>(p);
        return;
      }
      if (nd == 2) gemm_glds_kernel<BM, BN, 2, AMODE, CMODE, TC, H><<<grid, 256, 0, st>>>(p);
      else if (nd == 3) gemm_glds_kernel<BM, BN, (NMAX >= 3 ? 3 : 2), AMODE, CMODE, TC, H><<<grid, 256, 0, st>>>(p);
      else if (nd == 4 || NMAX < 5) gemm_glds_kernel<BM, BN, (NMAX >= 4 ? 4 : 2), AMODE, CMODE, TC, H><<<grid, 256, 0, st>>>(p);
      else gemm_glds_kernel<BM, BN, (NMAX >= 5 ? 5 : 2), AMODE, CMODE, TC, H><<<grid, 256, 0, st>>>(p);
      return;
    }
  }
  if constexpr (BN <= 256) {  // the register-staged tiles (a 64 x 512 one would not fit its double buffer in LDS)
    if (p.K <= 32) gemm_bf16_kernel<BM, BN, 32, AMODE, CMODE, TA, TC, H><<<grid, 256, 0, st>>>(p);
    else gemm_bf16_kernel<BM, BN, 64, AMODE, CMODE, TA, TC, H><<<grid, 256, 0, st>>>(p);
  }
}

// largest tile (no wider than N or taller than M, rounded up to 64) that still gives >= 512 blocks (2 per CU; with the
// 8-wave DMA tiles: 1024 with the register-staged 4-wave kernel measured best); otherwise 64x64, the most blocks.
#ifdef NBP_GEMM_MINBLK  // probe builds only (scripts/build_probe.py MINBLK=...)
constexpr long GEMM_MINBLK = NBP_GEMM_MINBLK;
#else
constexpr long GEMM_MINBLK = 512;
#endif

// 256 x 256 tiles on 8 waves (2 x 4, 128 x 64 each; two-pass epilogue) for the 3x3 implicit-GEMM convs with N >= 256
// while the grid still has >= 256 workgroups.  Measured (scripts/conv_micro.py, fp16, bs 8): +34-39 % on the 128^2 x
// 256 and 64^2 x 512 VGG layers (629 -> 842, 659 -> 913 TFLOP/s; bitwise equal: the same MFMA sequence per output
// element).  The other 256-row shapes (256 x 64, 256 x 128, 32-wide K-tiles) were measured neutral or slower
//  and removed.

template <int AMODE, int CMODE, typename TA, typename TC, typename H>
bool launch_conv_big(const GemmPB& p, hipStream_t st) {
  if constexpr (sizeof(TA) == 2 && AMODE == AM_IM2COL && CMODE != CM_LNBWD && CMODE != CM_CHANDOT &&
                CMODE != CM_RESLN) {
    const int ns = glds_depth();
    if ((ns >= 0 && ns < 2) || p.K <= 32 || p.ldb % 8 || p.cs % 8) return false;
    if (p.N >= 256 && (long)cdiv(p.M, 256) * cdiv(p.N, 256) >= 256) {
      // 256 x 256 tiles on 2 x 4 waves (128 x 64 each): twice the MFMA work per staged byte of the 128 x 128 tile
      const dim3 grid(cdiv(p.M, 256), cdiv(p.N, 256));
      gemm_glds_kernel<256, 256, 2, AMODE, CMODE, TC, H, 4, 2><<<grid, 512, 0, st>>>(p);
      return true;
    }
  }
  return false;
}

template <int AMODE, int CMODE, typename TA, typename TC, typename H>
void dispatch(const GemmPB& p, hipStream_t st) {
  if (launch_conv_big<AMODE, CMODE, TA, TC, H>(p, st)) return;
  if constexpr (CMODE == CM_CHANDOT) {  // its partial-sum layout is per 64-row tile
    launch<64, 64, AMODE, CMODE, TA, TC, H>(p, st);
  } else {
    auto blocks = [&](int bm, int bn) { return (long)cdiv(p.M, bm) * cdiv(p.N, bn); };
    const bool n128 = p.N > 64, m128 = p.M > 64;
    const long mb = GEMM_MINBLK;
    if (m128 && n128 && blocks(128, 128) >= mb) launch<128, 128, AMODE, CMODE, TA, TC, H>(p, st);
    else if (m128 && blocks(128, 64) >= mb) launch<128, 64, AMODE, CMODE, TA, TC, H>(p, st);
    else if (n128 && blocks(64, 128) >= mb) launch<64, 128, AMODE, CMODE, TA, TC, H>(p, st);
    else launch<64, 64, AMODE, CMODE, TA, TC, H>(p, st);
  }
}


template <typename TA, typename TC, typename H>
int dispatch_modes(const GemmPB& p, int a_mode, int c_mode, hipStream_t st) {
  if (a_mode == AM_PLAIN && c_mode == CM_PLAIN) dispatch<AM_PLAIN, CM_PLAIN, TA, TC, H>(p, st);
  else if (a_mode == AM_SCALE && c_mode == CM_PLAIN) dispatch<AM_SCALE, CM_PLAIN, TA, TC, H>(p, st);
  else if (a_mode == AM_S2D && c_mode == CM_PLAIN) dispatch<AM_S2D, CM_PLAIN, TA, TC, H>(p, st);
  else if (a_mode == AM_PLAIN && c_mode == CM_D2S) dispatch<AM_PLAIN, CM_D2S, TA, TC, H>(p, st);
  else if (a_mode == AM_PLAIN && c_mode == CM_SG) dispatch<AM_PLAIN, CM_SG, TA, TC, H>(p, st);
  else if (a_mode == AM_SCALE && c_mode == CM_SGBWD) dispatch<AM_SCALE, CM_SGBWD, TA, TC, H>(p, st);
  else if (a_mode == AM_PLAIN && c_mode == CM_SGBWD) dispatch<AM_PLAIN, CM_SGBWD, TA, TC, H>(p, st);
  else if (a_mode == AM_PLAIN && c_mode == CM_CHANDOT) dispatch<AM_PLAIN, CM_CHANDOT, TA, TC, H>(p, st);
  else {
    set_error("nbp_gemm_bf16: unsupported mode combination");
    return NBP_ERR_ARG;
  }
  return NBP_OK;
}

}  // namespace
