// fp32 MFMA GEMMs for every channel contraction of NAFNet on NHWC activations:
//   the NAFBlock 1x1 convs conv1/conv3/conv4/conv5 (NAFNet_arch.py:31-48), the 2x2/s2 down conv (:106-108,
//   as a GEMM over a space-to-depth gather), the 1x1 up conv + PixelShuffle(2) (:117-122, as a GEMM whose
//   epilogue scatters depth-to-space and adds the skip, :148-149), and their dgrad / wgrad.
// v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulation (one rounding per fma).
#include <type_traits>
#include <cstdint>
#include <vector>

#include <algorithm>

#include "nbp_common.h"

using namespace nbp;

namespace {

enum { AM_PLAIN = 0, AM_S2D = 1, AM_SCALE = 2, AM_CONV = 3 };
enum { CM_PLAIN = 0, CM_D2S = 1, CM_RELU = 2, CM_MASK = 3 };

struct GemmP {
  const float* A;
  long lda;
  const float* a_scale;
  int rows_per_img;
  const float* B;
  long ldb;
  float* C;
  long ldc;
  int M, N, K;
  int gh, gw, cs;  // S2D/D2S geometry: low-res grid gh x gw, cs channels per sub-position of the 2x map
  const float* bias;
  const float* R;
  const float* rscale;
  float* pre;
  // AM_CONV (implicit-GEMM KH x KW / stride conv over an NHWC map, zero padded): input ih x iw x cin, output grid
  // gh x gw (rows m = (b, oi, oj)), K index = (ki * kw + kj) * cin + c
  int ih, iw, cin, kh, kw, stride, pad;
};

// offset of element (m, kq*4 .. +3) of a space-to-depth view of a 2x-resolution NHWC map
__device__ __forceinline__ long s2d_off(int m, int k, int gh, int gw, int cs) {
  const int per = gh * gw;
  const int b = m / per, rem = m - b * per;
  const int i = rem / gw, j = rem - i * gw;
  const int q = k / cs, c = k - q * cs;
  const int kh = q >> 1, kw = q & 1;
  return ((long)(b * 2 * gh + 2 * i + kh) * (2 * gw) + 2 * j + kw) * cs + c;
}

template <int BM, int BN, bool B_NK, int AMODE, int CMODE>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmP p) {
  constexpr int BK = 32, LS = BK + 1;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int A_IT = BM / 32, B_IT = BN / 32;  // float4 loads per thread per K-tile
  __shared__ float As[BM * LS];
  __shared__ float Bs[BN * LS];
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

  float4 ra[A_IT], rb[B_IT];
  // AM_CONV: each thread's A rows are fixed over the K loop: image origin and top-left input tap of its rows
  long cbase[AM_CONV == AMODE ? A_IT : 1];
  int ci0[AM_CONV == AMODE ? A_IT : 1], cj0[AM_CONV == AMODE ? A_IT : 1];
  if (AMODE == AM_CONV) {
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int m = m0 + ((tid + it * 256) >> 3);
      const int per = p.gh * p.gw, b = m / per, rem = m - b * per, oi = rem / p.gw, oj = rem - oi * p.gw;
      cbase[it] = (long)b * p.ih * p.iw * p.cin;
      ci0[it] = oi * p.stride - p.pad;
      cj0[it] = oj * p.stride - p.pad;
    }
  }

  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int idx = tid + it * 256;
      const int r = idx >> 3, kq = idx & 7;
      const int m = m0 + r, k = k0 + kq * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M && k < K) {
        if (AMODE == AM_CONV) {
          const int tap = k / p.cin, c = k - tap * p.cin, ki = tap / p.kw, kj = tap - ki * p.kw;
          const int ii = ci0[it] + ki, jj = cj0[it] + kj;
          if (ii >= 0 && ii < p.ih && jj >= 0 && jj < p.iw)
            v = ld4(p.A + cbase[it] + ((long)ii * p.iw + jj) * p.cin + c);
        } else if (AMODE == AM_S2D) v = ld4(p.A + s2d_off(m, k, p.gh, p.gw, p.cs));
        else v = ld4(p.A + (long)m * p.lda + k);
        if (AMODE == AM_SCALE) v = v * ld4(p.a_scale + (long)(m / p.rows_per_img) * K + k);
      }
      ra[it] = v;
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int idx = tid + it * 256;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (B_NK) {
        const int r = idx >> 3, kq = idx & 7;
        const int n = n0 + r, k = k0 + kq * 4;
        if (n < N && k < K) v = ld4(p.B + (long)n * p.ldb + k);
      } else {
        const int kr = idx / (BN / 4), nq = idx % (BN / 4);
        const int k = k0 + kr, n = n0 + nq * 4;
        if (k < K && n < N) v = ld4(p.B + (long)k * p.ldb + n);
      }
      rb[it] = v;
    }
  };
  auto store_tiles = [&]() {
#pragma unroll
    for (int it = 0; it < A_IT; ++it) {
      const int idx = tid + it * 256;
      const int r = idx >> 3, kq = idx & 7;
      float* d = As + r * LS + kq * 4;
      d[0] = ra[it].x; d[1] = ra[it].y; d[2] = ra[it].z; d[3] = ra[it].w;
    }
#pragma unroll
    for (int it = 0; it < B_IT; ++it) {
      const int idx = tid + it * 256;
      if (B_NK) {
        const int r = idx >> 3, kq = idx & 7;
        float* d = Bs + r * LS + kq * 4;
        d[0] = rb[it].x; d[1] = rb[it].y; d[2] = rb[it].z; d[3] = rb[it].w;
      } else {
        const int kr = idx / (BN / 4), nq = idx % (BN / 4);
        float* d = Bs + (nq * 4) * LS + kr;
        d[0] = rb[it].x; d[LS] = rb[it].y; d[2 * LS] = rb[it].z; d[3 * LS] = rb[it].w;
      }
    }
  };

  const int nk = (K + BK - 1) / BK;
  load_tiles(0);
  store_tiles();
  __syncthreads();
  const int arow = wm * (BM / 2) + (lane & 31);
  const int brow = wn * (BN / 2) + (lane & 31);
  const int kh = lane >> 5;
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) load_tiles((t + 1) * BK);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[(arow + i * 32) * LS + kk + kh];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[(brow + j * 32) * LS + kk + kh];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (t + 1 < nk) {
      store_tiles();
      __syncthreads();
    }
  }

  // epilogue: C/D map of 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn * (BN / 2) + j * 32 + (lane & 31);
      if (col >= N) continue;
      const float bcol = p.bias ? p.bias[col] : 0.f;
      const float scol = p.rscale ? p.rscale[col] : 1.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= M) continue;
        long off;
        if (CMODE == CM_D2S) off = s2d_off(row, col, p.gh, p.gw, p.cs);
        else off = (long)row * p.ldc + col;
        float v = acc[i][j][r] + bcol;
        if (CMODE == CM_RELU) {
          p.C[off] = fmaxf(v, 0.f);
          continue;
        }
        if (CMODE == CM_MASK) {  // y = acc where R > 0 (the previous post-ReLU map), no bias
          p.C[off] = p.R[off] > 0.f ? acc[i][j][r] : 0.f;
          continue;
        }
        if (p.pre) p.pre[off] = v;
        if (p.R) v = p.R[off] + scol * v;
        p.C[off] = v;
      }
    }
}

// ---------------------------------------------------------------- weight gradient: dW[n][k] = sum_m G(m,n) X(m,k)
struct WgradP {
  const void* G;
  long ldg;
  const void* X;
  long ldx;
  const float* x_scale;
  int rows_per_img;
  int M, N, K;
  int gh, gw, cs_g, cs_x;
  float* slab;    // [S][N][K]
  float* slab_b;  // [S][N] (column sums of G) or null
  int chunk;
};

template <int GMODE, int XMODE, typename T>
__global__ __launch_bounds__(256) void wgrad_f32_kernel(WgradP p) {
  const T* G = reinterpret_cast<const T*>(p.G);
  const T* X = reinterpret_cast<const T*>(p.X);
  constexpr int RM = 32, TNW = 64, TKW = 64, LS = 68;
  __shared__ float Gs[RM * LS];
  __shared__ float Xs[RM * LS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = blockIdx.x * TNW, k0 = blockIdx.y * TKW, s = blockIdx.z;
  const int mb = s * p.chunk;
  const int me = min(p.M, mb + p.chunk);
  const bool do_b = p.slab_b && blockIdx.y == 0;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float bsum = 0.f;
  float4 rg[2], rx[2];
  auto load = [&](int m0) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + it * 256;
      const int r = idx >> 4, q = idx & 15;
      const int m = m0 + r;
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f), x = g;
      const int n = n0 + q * 4, k = k0 + q * 4;
      if (m < me) {
        if (n < p.N) {
          if (GMODE == AM_S2D) g = ldq(G + s2d_off(m, n, p.gh, p.gw, p.cs_g));
          else g = ldq(G + (long)m * p.ldg + n);
        }
        if (k < p.K) {
          if (XMODE == AM_S2D) x = ldq(X + s2d_off(m, k, p.gh, p.gw, p.cs_x));
          else x = ldq(X + (long)m * p.ldx + k);
          if (XMODE == AM_SCALE) x = x * ld4(p.x_scale + (long)(m / p.rows_per_img) * p.K + k);
        }
      }
      rg[it] = g;
      rx[it] = x;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int idx = tid + it * 256;
      const int r = idx >> 4, q = idx & 15;
      st4(Gs + r * LS + q * 4, rg[it]);
      st4(Xs + r * LS + q * 4, rx[it]);
    }
  };
  const int kh = lane >> 5;
  if (mb < me) {
    load(mb);
    store();
    __syncthreads();
    for (int m0 = mb; m0 < me; m0 += RM) {
      const bool more = m0 + RM < me;
      if (more) load(m0 + RM);
#pragma unroll
      for (int kk = 0; kk < RM; kk += 2) {
        const float a = Gs[(kk + kh) * LS + wn * 32 + (lane & 31)];
        const float b = Xs[(kk + kh) * LS + wk * 32 + (lane & 31)];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      }
      if (do_b && tid < TNW) {
#pragma unroll 8
        for (int r = 0; r < RM; ++r) bsum += Gs[r * LS + tid];
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = n0 + wn * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int k = k0 + wk * 32 + (lane & 31);
    if (n < p.N && k < p.K) p.slab[((long)s * p.N + n) * p.K + k] = acc[r];
  }
  if (do_b && tid < TNW && n0 + tid < p.N) p.slab_b[(long)s * p.N + n0 + tid] = bsum;
}

// bf16 storage: v_mfma_f32_32x32x16_bf16 with both operands read transposed from natural row-major LDS images by
// ds_read_b64_tr_b16 (the reduction index m is the ROW of G and X).  Lane 4q+p of a 16-lane group supplies the
// address of row q, columns 4p..4p+3 of a 4x16 block; lane i receives column i of the 4 rows.  Two reads give the
// 8 consecutive-m values of one fragment.  Rows are padded to 96 elements (192 B) so the four rows x two groups of
// a half-wave hit 64 distinct banks.
// RM = 64: 64-row stages -- twice the loads in flight per stage and half the barrier pairs; the
// MFMA and bias-sum order over the rows is unchanged (bitwise equal to RM = 32)
template <int GMODE, int XMODE, typename H, int RM = 32>
__global__ __launch_bounds__(256) void wgrad_bf16_kernel(WgradP p) {
  constexpr int TNW = 64, TKW = 64, LS = 96, NR = RM / 32;
  __shared__ __attribute__((aligned(16))) H Gs[RM * LS];
  __shared__ __attribute__((aligned(16))) H Xs[RM * LS];
  const H* G = reinterpret_cast<const H*>(p.G);
  const H* X = reinterpret_cast<const H*>(p.X);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = blockIdx.x * TNW, k0 = blockIdx.y * TKW, s = blockIdx.z;
  const int mb = s * p.chunk;
  const int me = min(p.M, mb + p.chunk);
  const bool do_b = p.slab_b && blockIdx.y == 0;
  floatx16 acc, tot;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = tot[r] = 0.f;
  float bsum = 0.f;
  // XMODE 3 = AM_SCALE with rows_per_img % 32 == 0: the MFMAs run on the unscaled X and each image's partial sum
  // is scaled by its column factor in fp32 when the 32-row stages move on to the next image (no per-element rescale)
  int cur_img = mb / p.rows_per_img;
  auto fold = [&](int im) {
    const int kk = k0 + wk * 32 + (lane & 31);
    const float sc = kk < p.K ? p.x_scale[(long)im * p.K + kk] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      tot[r] = fmaf(acc[r], sc, tot[r]);
      acc[r] = 0.f;
    }
  };
  // loader: NR 16-byte chunks of G and of X per thread: rows tid >> 3 (+ 32 i), 8 columns at (tid & 7) * 8
  const int lr = tid >> 3, lc = (tid & 7) * 8;
  vec_t<H, 8> rg[NR], rx[NR];
  auto load = [&](int m0) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = m0 + lr + 32 * i;
#pragma unroll
      for (int j = 0; j < 8; ++j) rg[i][j] = rx[i][j] = (H)0.f;
      if (m < me) {
        const int n = n0 + lc, k = k0 + lc;
        if (n < p.N) {
          const long off = GMODE == AM_S2D ? s2d_off(m, n, p.gh, p.gw, p.cs_g) : (long)m * p.ldg + n;
          rg[i] = *reinterpret_cast<const vec_t<H, 8>*>(G + off);
        }
        if (k < p.K) {
          const long off = XMODE == AM_S2D ? s2d_off(m, k, p.gh, p.gw, p.cs_x) : (long)m * p.ldx + k;
          rx[i] = *reinterpret_cast<const vec_t<H, 8>*>(X + off);
          if (XMODE == AM_SCALE) {
            const float* sc = p.x_scale + (long)(m / p.rows_per_img) * p.K + k;
#pragma unroll
            for (int j = 0; j < 8; ++j) rx[i][j] = (H)((float)rx[i][j] * sc[j]);
          }
        }
      }
    }
  };
  auto store_to = [&](H* gs, H* xs) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      *reinterpret_cast<vec_t<H, 8>*>(gs + (lr + 32 * i) * LS + lc) = rg[i];
      *reinterpret_cast<vec_t<H, 8>*>(xs + (lr + 32 * i) * LS + lc) = rx[i];
    }
  };
  auto store = [&]() { store_to(Gs, Xs); };
  // tr-read addressing (see header comment)
  const int grp = lane >> 4, gi = lane & 15, q = gi >> 2, pp = gi & 3, h = lane >> 5;
  const int gcol = wn * 32 + 16 * (grp & 1) + 4 * pp;
  const int xcol = wk * 32 + 16 * (grp & 1) + 4 * pp;
  if (mb < me) {
    load(mb);
    store();
    __syncthreads();
    for (int m0 = mb; m0 < me; m0 += RM) {
      const bool more = m0 + RM < me;
      if (more) load(m0 + RM);
      if constexpr (XMODE == 3) {
        const int im = m0 / p.rows_per_img;
        if (im != cur_img) {
          fold(cur_img);
          cur_img = im;
        }
      }
#pragma unroll
      for (int ks = 0; ks < RM; ks += 16) {
        vec_t<H, 8> a, b;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int row = ks + 8 * h + 4 * t + q;
          const vec_t<H, 4> va = ds_read_tr16<H>(Gs + row * LS + gcol);
          const vec_t<H, 4> vb = ds_read_tr16<H>(Xs + row * LS + xcol);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a[4 * t + j] = va[j];
            b[4 * t + j] = vb[j];
          }
        }
        acc = mfma32x32x16(a, b, acc);
      }
      if (do_b && tid < TNW) {
#pragma unroll 8
        for (int r = 0; r < RM; ++r) bsum += (float)Gs[r * LS + tid];
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
    }
  }
  if constexpr (XMODE == 3) {
    if (mb < me) fold(cur_img);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = n0 + wn * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int k = k0 + wk * 32 + (lane & 31);
    if (n < p.N && k < p.K) p.slab[((long)s * p.N + n) * p.K + k] = XMODE == 3 ? tot[r] : acc[r];
  }
  if (do_b && tid < TNW && n0 + tid < p.N) p.slab_b[(long)s * p.N + n0 + tid] = bsum;
}

// Narrow 16-bit weight gradient with the whole N x K output in one workgroup (N, K in {32, 64, 128}, at most 8 output
// tiles of 32 x 32: the level-0 / 1 NAFBlock 1x1 convs with plain or per-image-scaled X, and the level-0 / 1 down /
// up convs with the space-to-depth gather of X / G).  Against the 64 x 64 tiles above:
//  * every operand row is read once (they read X once per 64-column n-tile: 1.33x the bytes at N = 128);
//  * 1024 threads = 4 row groups of 4 waves, each group with its own LDS stage, taking the split's 64-row stages g,
//    g + 4, ...; the groups' partials are combined in LDS in a fixed order, so a split (and its fp32 slab) covers 4x
//    the rows at the same 16 waves per CU (one workgroup per CU);
//  * below four 32 x 32 output tiles the waves sharing a tile split its 16-row k-steps instead of idling.
// Fragments come transposed from 96-element LDS rows by ds_read_b64_tr_b16 as in wgrad_bf16_kernel.
template <int GMODE, int XMODE, typename H, int NT, int KT>
__global__ __launch_bounds__(1024) void wgrad_narrow_full(WgradP p) {
  static_assert(XMODE == AM_PLAIN || XMODE == 3 || XMODE == AM_S2D, "wgrad_narrow_full: plain, scaled or S2D X");
  static_assert(GMODE == AM_PLAIN || GMODE == AM_S2D, "wgrad_narrow_full: plain or S2D G");
  static_assert(NT * KT <= 8, "wgrad_narrow_full: at most 8 output tiles");
  constexpr int N = 32 * NT, K = 32 * KT, RG = 4, RM = 64, LS = 96;
  constexpr int NG = (N + 63) / 64, NX = (K + 63) / 64;      // 64-column G / X panels
  constexpr int PANEL = RM * LS;                             // 16-bit elements per panel
  constexpr int STAGE_BYTES = (NG + NX) * PANEL * (int)sizeof(H);
  constexpr int T = NT * KT;                                 // 32 x 32 output tiles
  constexpr int TW = T < 4 ? T : 4;                          // tiles a group's 4 waves work on at once
  constexpr int TPW = T > 4 ? T / 4 : 1;                     // tiles per wave
  constexpr int KSPLIT = 4 / TW;                             // waves sharing a tile (its k-steps split)
  constexpr int RED_BYTES = (RG * 4 * TPW * 1024 + RG * N) * 4;
  constexpr int SMEM = RG * STAGE_BYTES > RED_BYTES ? RG * STAGE_BYTES : RED_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, g = tid >> 8, gt = tid & 255, lane = tid & 63, w = gt >> 6;
  H* Gs = reinterpret_cast<H*>(smem + g * STAGE_BYTES);
  H* Xs = Gs + NG * PANEL;
  const H* G = reinterpret_cast<const H*>(p.G);
  const H* X = reinterpret_cast<const H*>(p.X);
  const int s = blockIdx.x;
  const int mb = s * p.chunk, me = min(p.M, mb + p.chunk);
  const bool do_b = p.slab_b != nullptr;
  const int ksub = w / TW;
  int tn[TPW], tk[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = T >= 4 ? w + 4 * j : w % TW;
    tn[j] = t / KT;
    tk[j] = t % KT;
  }
  floatx16 acc[TPW], tot[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = tot[j][r] = 0.f;
  float bsum = 0.f;
  int cur_img = -1;
  auto fold = [&](int im) {  // XMODE 3: each image's partial scaled by its column factors
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const float sc = p.x_scale[(long)im * K + tk[j] * 32 + (lane & 31)];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        tot[j][r] = fmaf(acc[j][r], sc, tot[j][r]);
        acc[j][r] = 0.f;
      }
    }
  };
  // loader: 8-element chunks, row-major over the stage (consecutive threads along a row, rows contiguous)
  constexpr int GC = RM * N / 8 / 256, XC = RM * K / 8 / 256;
  vec_t<H, 8> rg[GC], rx[XC];
  auto load = [&](int m0) {
#pragma unroll
    for (int i = 0; i < GC; ++i) {
      const int c = gt + 256 * i, m = m0 + c / (N / 8), col = (c % (N / 8)) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) rg[i][e] = (H)0.f;
      if (m < me)
        rg[i] = *reinterpret_cast<const vec_t<H, 8>*>(
            G + (GMODE == AM_S2D ? s2d_off(m, col, p.gh, p.gw, p.cs_g) : (long)m * p.ldg + col));
    }
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int c = gt + 256 * i, m = m0 + c / (K / 8), col = (c % (K / 8)) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) rx[i][e] = (H)0.f;
      if (m < me)
        rx[i] = *reinterpret_cast<const vec_t<H, 8>*>(
            X + (XMODE == AM_S2D ? s2d_off(m, col, p.gh, p.gw, p.cs_x) : (long)m * p.ldx + col));
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < GC; ++i) {
      const int c = gt + 256 * i, row = c / (N / 8), col = (c % (N / 8)) * 8;
      *reinterpret_cast<vec_t<H, 8>*>(Gs + (col / 64) * PANEL + row * LS + col % 64) = rg[i];
    }
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      const int c = gt + 256 * i, row = c / (K / 8), col = (c % (K / 8)) * 8;
      *reinterpret_cast<vec_t<H, 8>*>(Xs + (col / 64) * PANEL + row * LS + col % 64) = rx[i];
    }
  };
  const int grp = lane >> 4, gi = lane & 15, q = gi >> 2, pp = gi & 3, h = lane >> 5;
  const int cofs = 16 * (grp & 1) + 4 * pp;
  const int nst = mb < me ? (me - mb + RM - 1) / RM : 0;  // the split's stages; group g takes g, g + RG, ...
  const int niter = (nst + RG - 1) / RG;                   // (block-uniform: every barrier is reached by all)
  if (mb + g * RM < me) load(mb + g * RM);
  for (int i = 0; i < niter; ++i) {
    const int ms = mb + (i * RG + g) * RM;
    const bool valid = ms < me;
    if (valid) {
      if constexpr (XMODE == 3) {
        const int im = ms / p.rows_per_img;
        if (im != cur_img) {
          if (cur_img >= 0) fold(cur_img);
          cur_img = im;
        }
      }
      store();
    }
    __syncthreads();
    if (ms + RG * RM < me) load(ms + RG * RM);
    if (valid) {
#pragma unroll
      for (int kq = 0; kq < 4 / KSPLIT; ++kq) {
        const int ks = (ksub + KSPLIT * kq) * 16;
#pragma unroll
        for (int j = 0; j < TPW; ++j) {
          const H* gp = Gs + ((tn[j] * 32) / 64) * PANEL + (tn[j] * 32) % 64 + cofs;
          const H* xp = Xs + ((tk[j] * 32) / 64) * PANEL + (tk[j] * 32) % 64 + cofs;
          vec_t<H, 8> a, b;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int row = ks + 8 * h + 4 * t + q;
            const vec_t<H, 4> va = ds_read_tr16<H>(gp + row * LS);
            const vec_t<H, 4> vb = ds_read_tr16<H>(xp + row * LS);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              a[4 * t + e] = va[e];
              b[4 * t + e] = vb[e];
            }
          }
          acc[j] = mfma32x32x16(a, b, acc[j]);
        }
      }
      if (do_b && gt < N) {
        const H* col = Gs + (gt / 64) * PANEL + gt % 64;
#pragma unroll 8
        for (int r = 0; r < RM; ++r) bsum += (float)col[r * LS];
      }
    }
    __syncthreads();
  }
  if constexpr (XMODE == 3) {
    if (cur_img >= 0) fold(cur_img);
  }
  // partials through LDS (the stages are dead after the loop's last barrier), combined in a fixed order: row group,
  // then the waves sharing a tile in k-step order
  float* red = reinterpret_cast<float*>(smem);
  float* redb = red + RG * 4 * TPW * 1024;
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int nl = (r & 3) + 8 * (r >> 2) + 4 * h, kl = lane & 31;
      red[((g * 4 + w) * TPW + j) * 1024 + nl * 32 + kl] = XMODE == 3 ? tot[j][r] : acc[j][r];
    }
  if (do_b && gt < N) redb[g * N + gt] = bsum;
  __syncthreads();
  for (int e = tid; e < N * K; e += 1024) {
    const int n = e / K, k = e % K, t = (n / 32) * KT + k / 32, off = (n % 32) * 32 + k % 32;
    float v = 0.f;
#pragma unroll
    for (int gg = 0; gg < RG; ++gg)
#pragma unroll
      for (int ku = 0; ku < KSPLIT; ++ku) {
        const int wv = T >= 4 ? t % 4 : t + TW * ku, slot = T >= 4 ? t / 4 : 0;
        v += red[((gg * 4 + wv) * TPW + slot) * 1024 + off];
      }
    p.slab[(long)s * N * K + e] = v;
  }
  if (do_b && tid < N) p.slab_b[(long)s * N + tid] = ((redb[tid] + redb[N + tid]) + redb[2 * N + tid]) + redb[3 * N + tid];
}

// splits of the full-width narrow weight gradient: one workgroup (16 waves) per CU, >= 512 rows per split
int wgrad_full_splits(int M) {
  const int s = cdiv(M, 512);
  return s < 1 ? 1 : (s > 256 ? 256 : s);
}

// NBP_WGRAD_FULL=0: the 64 x 64-tile narrow weight gradient instead (A/B)
bool wgrad_full_enabled() {
  static const bool on = [] {
    const char* e = getenv("NBP_WGRAD_FULL");
    return !e || atoi(e) != 0;
  }();
  return on;
}

template <typename H, int XM>
void launch_wgrad_full(const WgradP& p, int S_, hipStream_t st) {
  const int N = p.N, K = p.K;
  if (N == 128 && K == 64) {
    if constexpr (XM == AM_PLAIN) wgrad_narrow_full<AM_PLAIN, XM, H, 4, 2><<<S_, 1024, 0, st>>>(p);  // (scaled: spills)
  } else if (N == 128) wgrad_narrow_full<AM_PLAIN, XM, H, 4, 1><<<S_, 1024, 0, st>>>(p);
  else if (N == 64 && K == 64) wgrad_narrow_full<AM_PLAIN, XM, H, 2, 2><<<S_, 1024, 0, st>>>(p);
  else if (N == 64) wgrad_narrow_full<AM_PLAIN, XM, H, 2, 1><<<S_, 1024, 0, st>>>(p);
  else if (K == 64) wgrad_narrow_full<AM_PLAIN, XM, H, 1, 2><<<S_, 1024, 0, st>>>(p);
  else wgrad_narrow_full<AM_PLAIN, XM, H, 1, 1><<<S_, 1024, 0, st>>>(p);
}

// the down conv (X gathered, N 64 x K 128) and up conv (G gathered, N 128 x K 64) gradients of levels 0 / 1
template <typename H>
void launch_wgrad_full_s2d(const WgradP& p, bool g_s2d, int S_, hipStream_t st) {
  if (g_s2d) wgrad_narrow_full<AM_S2D, AM_PLAIN, H, 4, 2><<<S_, 1024, 0, st>>>(p);
  else wgrad_narrow_full<AM_PLAIN, AM_S2D, H, 2, 4><<<S_, 1024, 0, st>>>(p);
}

// bf16 weight gradient for the wide layers (N, K multiples of 128: NAFBlock 1x1 convs at C >= 128): a 128 x 128
// output tile per workgroup, each wave a 64 x 64 quadrant (2 x 2 MFMA tiles of 32 x 32 x 16), 64-row stages
// (16 MFMAs per wave between barrier pairs, 8x the old 64 x 64 tile's), next stage prefetched into registers.
// Each operand tile lives in LDS as two 64-column panels with the conflict-free 96-element rows of
// wgrad_bf16_kernel, read transposed by ds_read_b64_tr_b16.  Bias (column sums of G) from the loader's registers.
constexpr int WIDE_LDS = 4 * 64 * 96;  // 16-bit elements: G panels 0, 1; X panels 2, 3 (64 rows x 96)

template <int XMODE, typename H>
__device__ __forceinline__ void wgrad_wide_tile(const WgradP& p, int bx, int by, int bz, H* lds) {
  constexpr int RM = 64, LS = 96, PAN = RM * LS;
  const H* G = reinterpret_cast<const H*>(p.G);
  const H* X = reinterpret_cast<const H*>(p.X);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = bx * 128, k0 = by * 128, s = bz;
  const int mb = s * p.chunk;
  const int me = min(p.M, mb + p.chunk);
  const bool do_b = p.slab_b && by == 0;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float bs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bs[i] = 0.f;
  // loader: 16-byte chunk cc of rows lrow + 16 j (j < 4) for both operands
  const int lrow = tid >> 4, cc = tid & 15, pan = cc >> 3, lcol = (cc & 7) * 8;
  vec_t<H, 8> rg[4], rx[4];
  auto load = [&](int m0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + lrow + 16 * j;
      if (m < me) {
        rg[j] = *reinterpret_cast<const vec_t<H, 8>*>(G + (long)m * p.ldg + n0 + cc * 8);
        rx[j] = *reinterpret_cast<const vec_t<H, 8>*>(X + (long)m * p.ldx + k0 + cc * 8);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rg[j][e] = rx[j][e] = (H)0.f;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *reinterpret_cast<vec_t<H, 8>*>(lds + pan * PAN + (lrow + 16 * j) * LS + lcol) = rg[j];
      *reinterpret_cast<vec_t<H, 8>*>(lds + (2 + pan) * PAN + (lrow + 16 * j) * LS + lcol) = rx[j];
      if (do_b) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bs[e] += (float)rg[j][e];
      }
    }
  };
  const int grp = lane >> 4, gi = lane & 15, q = gi >> 2, pp = gi & 3, h = lane >> 5;
  const int fcol = 16 * (grp & 1) + 4 * pp;
  const H* gpan = lds + wn * PAN;
  const H* xpan = lds + (2 + wk) * PAN;
  // AM_SCALE (X columns scaled per image; the launcher guarantees rows_per_img % 64 == 0, so no stage straddles two
  // images): the MFMAs run on the unscaled X and each image's partial sum is scaled in fp32 when the rows move on.
  constexpr int NT_ = XMODE == AM_SCALE ? 2 : 1;
  floatx16 tot[NT_][NT_];
#pragma unroll
  for (int i = 0; i < NT_; ++i)
#pragma unroll
    for (int j = 0; j < NT_; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) tot[i][j][r] = 0.f;
  int cur_img = mb / p.rows_per_img;
  auto fold = [&](int im) {
#pragma unroll
    for (int j = 0; j < NT_; ++j) {
      const float sc = p.x_scale[(long)im * p.K + k0 + wk * 64 + j * 32 + (lane & 31)];
#pragma unroll
      for (int i = 0; i < NT_; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          tot[i][j][r] = fmaf(acc[i][j][r], sc, tot[i][j][r]);
          acc[i][j][r] = 0.f;
        }
    }
  };
  if (mb < me) {
    load(mb);
    store();
    __syncthreads();
    for (int m0 = mb; m0 < me; m0 += RM) {
      const bool more = m0 + RM < me;
      if (more) load(m0 + RM);
      if constexpr (XMODE == AM_SCALE) {
        const int im = m0 / p.rows_per_img;
        if (im != cur_img) {
          fold(cur_img);
          cur_img = im;
        }
      }
#pragma unroll
      for (int ks = 0; ks < RM; ks += 16) {
        vec_t<H, 8> a[2], b[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int row = ks + 8 * h + 4 * t + q;
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const vec_t<H, 4> va = ds_read_tr16<H>(gpan + row * LS + i * 32 + fcol);
            const vec_t<H, 4> vb = ds_read_tr16<H>(xpan + row * LS + i * 32 + fcol);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              a[i][4 * t + e] = va[e];
              b[i][4 * t + e] = vb[e];
            }
          }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma32x32x16(a[i], b[j], acc[i][j]);
      }
      __syncthreads();
      if (more) {
        store();
        __syncthreads();
      }
    }
    if constexpr (XMODE == AM_SCALE) fold(cur_img);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int k = k0 + wk * 64 + j * 32 + (lane & 31);
        float v;
        if constexpr (XMODE == AM_SCALE) v = tot[i % NT_][j % NT_][r];
        else v = acc[i][j][r];
        p.slab[((long)s * p.N + n) * p.K + k] = v;
      }
  if (do_b) {  // 16 loader rows share a column chunk: fixed-order LDS combine
    float* red = reinterpret_cast<float*>(lds);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[lrow * 128 + cc * 8 + e] = bs[e];
    __syncthreads();
    if (tid < 128) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) t += red[r * 128 + tid];
      p.slab_b[(long)s * p.N + n0 + tid] = t;
    }
  }
}

// The same 128 x 128 tile with the operand panels staged by LDS-DMA into an NS-deep ring (NS - 1 stages in flight
// across the barriers, counted vmcnt, raw s_barrier): the register-staged tile above issues a stage's loads one stage
// ahead and its in-order vmcnt waits expose their latency every stage.  Panel image: 64 rows x 128 columns of 256 B,
// the 16-byte chunk c of row r at slot c ^ (4 (r & 3)) (permuted on the DMA source address), which keeps the
// ds_read_b64_tr_b16 fragment reads (4 rows x 8 column pieces per 32-lane group) conflict-free.  The per-image SCA
// scale of the stage's 128 X columns is DMA'd with the stage (a stage never straddles two images); the bias column
// sums of G are read back from the panel.  Same MFMA sequence per tile as wgrad_wide_tile (the bias sums are added
// in another order).
// WNW = 4: 256 x 128 output tiles on 8 waves (4 along N x 2 along K, each 64 x 64; the G panel rows are 512 B) --
// measured slower in the grouped weight gradients, no longer instantiated.
template <int NS, int XMODE, int WNW = 2>
constexpr int wide_glds_stage_bytes() { return 64 * 128 * WNW + 64 * 256 + (XMODE == AM_SCALE ? 512 : 0); }
template <int NS, int WNW = 2>
constexpr int wide_glds_lds_bytes() {
  return NS * wide_glds_stage_bytes<NS, AM_SCALE, WNW>() > 16 * 128 * 4 ? NS * wide_glds_stage_bytes<NS, AM_SCALE, WNW>()
                                                                        : 16 * 128 * 4;
}

// asm helpers of wgrad_wide_tile_glds: the 8 ds_read_b64_tr_b16 of one 16-row K step (rows KS + 4 t + lane part),
// fragment order [t * 4 + {Gi0, Gi1, Xi0, Xi1}]; a counted lgkmcnt wait that also ties the fragments to it (so no
// consumer is scheduled above the wait); and the step's 2 x 2 MFMAs.
template <int KS, int GRB = 256>  // GRB: G panel row bytes
__device__ __forceinline__ void wide_tr_reads(s16x4 (&f)[8], unsigned g0, unsigned g1, unsigned x0, unsigned x1) {
#define NBP_TR(dst, addr, off) asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "n"(off))
  NBP_TR(f[0], g0, KS * GRB);
  NBP_TR(f[1], g1, KS * GRB);
  NBP_TR(f[2], x0, KS * 256);
  NBP_TR(f[3], x1, KS * 256);
  NBP_TR(f[4], g0, (KS + 4) * GRB);
  NBP_TR(f[5], g1, (KS + 4) * GRB);
  NBP_TR(f[6], x0, (KS + 4) * 256);
  NBP_TR(f[7], x1, (KS + 4) * 256);
#undef NBP_TR
}
template <int N>
__device__ __forceinline__ void wide_tr_wait(s16x4 (&f)[8]) {
  asm volatile("s_waitcnt lgkmcnt(%8)"
               : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
               : "n"(N));
}
template <typename H>
__device__ __forceinline__ void wide_mfma(const s16x4 (&f)[8], floatx16 (&acc)[2][2], bool bias, floatx16 (&accb)[2]) {
  vec_t<H, 8> a[2], b[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const vec_t<H, 4> a0 = __builtin_bit_cast(vec_t<H, 4>, f[i]), a1 = __builtin_bit_cast(vec_t<H, 4>, f[4 + i]);
    const vec_t<H, 4> b0 = __builtin_bit_cast(vec_t<H, 4>, f[2 + i]), b1 = __builtin_bit_cast(vec_t<H, 4>, f[6 + i]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[i][e] = a0[e];
      a[i][4 + e] = a1[e];
      b[i][e] = b0[e];
      b[i][4 + e] = b1[e];
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = mfma32x32x16(a[i], b[j], acc[i][j]);
  if (bias) {  // column sums of G: the same A fragments against a ones B fragment (every output column = the sum)
    vec_t<H, 8> ones;
#pragma unroll
    for (int e = 0; e < 8; ++e) ones[e] = (H)1.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) accb[i] = mfma32x32x16(a[i], ones, accb[i]);
  }
}

// LW (loader waves): 8 waves -- waves 4..7 only issue the stage DMAs (the geometry of waves 0..3 above), waves 0..3
// only read fragments and multiply (the same MFMA sequence per output element: bitwise equal to LW = false).  Every
// wave of the 4-wave tile issued 8 1-KB DMA pieces per 64-row stage beside its 16 MFMAs; in one instruction stream
// the piece issue (60-185 cycles each among MFMAs, MI355X_MICROARCH.md 'LDS-DMA piece issue cost') and the MFMAs
// serialise.  Split, the loaders' issue overlaps the consumers' MFMAs on the same SIMDs.
template <int XMODE, typename H, int NS, int WNW = 2, bool LW = false>
__device__ __forceinline__ void wgrad_wide_tile_glds(const WgradP p, int bx, int by, int bz, unsigned char* smem) {
  constexpr int NWV = 2 * WNW, TNB = 64 * WNW;  // (compute) waves; output tile columns (N)
  constexpr int NDW = LW ? 4 : NWV;              // waves that issue the stage DMAs
  constexpr int GRB = 2 * TNB, RM = 64, PAN = RM * GRB, ST = wide_glds_stage_bytes<NS, XMODE, WNW>();
  constexpr int GRI = 1024 / GRB, GLPR = 64 / GRI;  // G rows per DMA instruction, lanes per G row
  constexpr int IG = RM / (GRI * NDW), IX = RM / (4 * NDW);  // DMA instructions per wave per stage (G, X)
  constexpr int GL = IG + IX + (XMODE == AM_SCALE && !LW ? 2 : 0);
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  static_assert(WNW == 2 || WNW == 4, "wave columns");
  const H* G = reinterpret_cast<const H*>(p.G);
  const H* X = reinterpret_cast<const H*>(p.X);
  const int tid = threadIdx.x, lane = tid & 63, wave_id = tid >> 6;
  // LW: waves NWV .. NWV + 3 load (DMA geometry index dwave), waves 0 .. NWV - 1 compute
  const bool loads = !LW || wave_id >= NWV, computes = !LW || wave_id < NWV;
  const int dwave = LW ? (wave_id >= NWV ? wave_id - NWV : 0) : wave_id;
  const int wave = wave_id;
  const int wn = wave >> 1, wk = wave & 1;
  const int n0 = bx * TNB, k0 = by * 128, s = bz;
  const int mb = s * p.chunk;
  const int me = min(p.M, mb + p.chunk);
  const bool do_b = p.slab_b && by == 0;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  constexpr int NT_ = XMODE == AM_SCALE ? 2 : 1;
  floatx16 tot[NT_][NT_];
#pragma unroll
  for (int i = 0; i < NT_; ++i)
#pragma unroll
    for (int j = 0; j < NT_; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) tot[i][j][r] = 0.f;
  // DMA geometry: G instruction j of this wave fills panel rows (IG wave + j) * GRI + lane / GLPR, physical slot
  // lane % GLPR; X instruction j rows (IX wave + j) * 4 + lane / 16, slot lane % 16; chunk c at slot c ^ 4 (r & 3)
  int grow_[IG], gcol_[IG], xrow_[IX], xcol_[IX];
#pragma unroll
  for (int j = 0; j < IG; ++j) {
    grow_[j] = (dwave * IG + j) * GRI + lane / GLPR;
    gcol_[j] = 8 * ((lane % GLPR) ^ (4 * (grow_[j] & 3)));
  }
#pragma unroll
  for (int j = 0; j < IX; ++j) {
    xrow_[j] = (dwave * IX + j) * 4 + (lane >> 4);
    xcol_[j] = 8 * ((lane & 15) ^ (4 * (xrow_[j] & 3)));
  }
  const int nst = mb < me ? (me - mb + RM - 1) / RM : 0;
  // the zero page's address in registers (laundered through asm: otherwise it is re-loaded from the GOT, with an
  // lgkmcnt(0) wait, at every use inside the loop)
  const void* zp = g_zero16;
  asm volatile("" : "+s"(zp));
  // running source pointers and rows of this lane's pieces (issue() is called for t = 0, 1, 2, ... in order): one
  // 64-bit add per piece and stage instead of a 64-bit multiply, and a select of the zero page past the chunk's end
  const H* gsrc[IG];
  const H* xsrc[IX];
  int grw[IG], xrw[IX];
#pragma unroll
  for (int j = 0; j < IG; ++j) {
    grw[j] = mb + grow_[j];
    gsrc[j] = G + (long)grw[j] * p.ldg + n0 + gcol_[j];
  }
#pragma unroll
  for (int j = 0; j < IX; ++j) {
    xrw[j] = mb + xrow_[j];
    xsrc[j] = X + (long)xrw[j] * p.ldx + k0 + xcol_[j];
  }
  const long gstep = (long)RM * p.ldg, xstep = (long)RM * p.ldx;
  auto issue = [&](int t) {
    unsigned char* st = smem + (t % NS) * ST;
#pragma unroll
    for (int j = 0; j < (IG > IX ? IG : IX); ++j) {  // (IG == IX == 4 at WNW 2: the original G / X interleave)
      if (j < IG) {
        glds16(grw[j] < me ? (const void*)gsrc[j] : zp, st + (dwave * IG + j) * 1024);
        grw[j] += RM;
        gsrc[j] += gstep;
      }
      if (j < IX) {
        glds16(xrw[j] < me ? (const void*)xsrc[j] : zp, st + PAN + (dwave * IX + j) * 1024);
        xrw[j] += RM;
        xsrc[j] += xstep;
      }
    }
    if constexpr (XMODE == AM_SCALE && !LW) {  // every wave DMAs the same 128 scales of the stage's image
      const float* sc = p.x_scale + (long)((mb + t * RM) / p.rows_per_img) * p.K + k0;
      glds4(sc + lane, st + PAN + RM * 256);
      glds4(sc + 64 + lane, st + PAN + RM * 256 + 256);
    }
  };
  // fragment reads: lane (grp, q, pp, h) reads row ks + 8h + 4t + q, logical column (wave half) + 32 i + fcol; in the
  // panel image that is byte row * 256 + 16 ((col / 8) ^ 4q) + 2 (col % 8).  The lane part is folded into four base
  // addresses (G / X, i = 0 / 1); the rows ks + 4t are immediate offsets.
  const int grp = lane >> 4, gi = lane & 15, q = gi >> 2, pp = gi & 3, h = lane >> 5;
  const int lx = 2 * (grp & 1) + (pp >> 1);  // chunk within the 4-chunk (32-column) group
  unsigned abase[2][2];                      // [G / X][i], relative to the stage
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    abase[0][i] = (8 * h + q) * GRB + ((4 * ((2 * wn + i) ^ q) + lx) << 4) + (pp & 1) * 8;
    abase[1][i] = PAN + (8 * h + q) * 256 + ((4 * ((2 * wk + i) ^ q) + lx) << 4) + (pp & 1) * 8;
  }
  const unsigned smem_lds = (unsigned)(size_t)(lds_void_t*)smem;
  // fragment sets: K steps 0 / 2 -> fa, 1 -> fc, 3 -> fb (the last K step multiplied under the next stage's first
  // reads)
  s16x4 fa[8], fb[8], fc[8];
  float cur_sc[2] = {0.f, 0.f};
  auto fold = [&]() {
#pragma unroll
    for (int j = 0; j < NT_; ++j)
#pragma unroll
      for (int i = 0; i < NT_; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          tot[i][j][r] = fmaf(acc[i][j][r], cur_sc[j], tot[i][j][r]);
          acc[i][j][r] = 0.f;
        }
  };
  // bias (column sums of G) on the MFMA pipe: waves wk == 0 of the by == 0 tiles
  const bool wb = do_b && wk == 0 && computes;
  floatx16 accb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) accb[i][r] = 0.f;

  // the stage loop per role (R: 0 = load and compute, 1 = load only, 2 = compute only): with loader waves the roles
  // are separate loops with the same barriers, so neither role's loop-carried registers are live in the other's
  auto run = [&](auto role) {
    constexpr int R = decltype(role)::value;
    constexpr bool RL = R != 2, RC = R != 1;
    if (RL) {
  #pragma unroll
      for (int t = 0; t < NS - 1; ++t)
        if (t < nst) issue(t);
    }
    // the stages of one image form an inner loop with no fold inside it (a conditional fold in the stage loop made the
    // compiler move all 64 accumulators between AGPRs and VGPRs every stage); AM_PLAIN: one segment
    for (int t = 0; t < nst;) {
      int tend = nst;
      if constexpr (XMODE == AM_SCALE) {
        const int im = (mb + t * RM) / p.rows_per_img;
        tend = min(nst, ((im + 1) * p.rows_per_img - mb + RM - 1) / RM);
        if (LW && RC) {  // the consumers have no DMA in flight: a plain load of the image's 128 scales
          const float* sc = p.x_scale + (long)im * p.K + k0 + wk * 64 + (lane & 31);
          cur_sc[0] = sc[0];
          cur_sc[1] = sc[32];
        }
      }
      const int tseg = t;
      for (; t < tend; ++t) {
        // retire stage t: the stages issued after it (at most NS - 2) stay in flight
        if (RL) {
          if (NS >= 4 && t + 2 < nst) wait_vm<2 * GL>();
          else if (NS >= 3 && t + 1 < nst) wait_vm<GL>();
          else wait_vm<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (RL && t + NS - 1 < nst) issue(t + NS - 1);
        if (!RC) continue;
        if constexpr (XMODE == AM_SCALE && !LW) {
          if (t == tseg) {  // (asm LDS reads: a plain load here would make the compiler drain the DMA ring first)
            const unsigned sa = smem_lds + (t % NS) * ST + PAN + RM * 256 + (wk * 64 + (lane & 31)) * 4;
            asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %2 offset:128\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(cur_sc[0]), "=&v"(cur_sc[1])
                         : "v"(sa));
          }
        }
        // the 8 tr-reads of K step ks + 16 are in flight while step ks is multiplied (asm: a builtin tr-read would make
        // the compiler drain the DMA ring, vmcnt(0), before it).  The stage's last K step (set fb) is multiplied after the
        // next stage's barrier, under that stage's first fragment reads (the same MFMA order per accumulator)
        const unsigned sb = smem_lds + (t % NS) * ST;
        const unsigned ga0 = sb + abase[0][0], ga1 = sb + abase[0][1], xa0 = sb + abase[1][0], xa1 = sb + abase[1][1];
        wide_tr_reads<0, GRB>(fa, ga0, ga1, xa0, xa1);
        wide_tr_reads<16, GRB>(fc, ga0, ga1, xa0, xa1);
        if (t != tseg) wide_mfma<H>(fb, acc, wb, accb);
        wide_tr_wait<8>(fa);
        wide_mfma<H>(fa, acc, wb, accb);
        wide_tr_reads<32, GRB>(fa, ga0, ga1, xa0, xa1);
        wide_tr_wait<8>(fc);
        wide_mfma<H>(fc, acc, wb, accb);
        wide_tr_reads<48, GRB>(fb, ga0, ga1, xa0, xa1);
        wide_tr_wait<8>(fa);
        wide_mfma<H>(fa, acc, wb, accb);
        wide_tr_wait<0>(fb);  // (every read of the slot done before the next barrier frees it)
      }
      if (RC && tend > tseg) wide_mfma<H>(fb, acc, wb, accb);
      if constexpr (XMODE == AM_SCALE)
        if (RC) fold();
    }
  };
  if constexpr (!LW) run(std::integral_constant<int, 0>{});
  else if (loads) run(std::integral_constant<int, 1>{});
  else run(std::integral_constant<int, 2>{});
  if (!computes) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int k = k0 + wk * 64 + j * 32 + (lane & 31);
        float v;
        if constexpr (XMODE == AM_SCALE) v = tot[i % NT_][j % NT_][r];
        else v = acc[i][j][r];
        p.slab[((long)s * p.N + n) * p.K + k] = v;
      }
  if (wb && (lane & 31) == 0)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        p.slab_b[(long)s * p.N + n0 + wn * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)] = accb[i][r];
}

template <int XMODE, typename H>
__global__ __launch_bounds__(256) void wgrad_bf16_wide(WgradP p) {
  __shared__ __attribute__((aligned(16))) H lds[WIDE_LDS];
  wgrad_wide_tile<XMODE, H>(p, blockIdx.x, blockIdx.y, blockIdx.z, lds);
}

template <int XMODE, typename H, int NS>
__global__ __launch_bounds__(256) void wgrad_bf16_wide_glds(WgradP p) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[wide_glds_lds_bytes<NS>()];
  wgrad_wide_tile_glds<XMODE, H, NS>(p, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

// Many independent wide weight gradients in one launch (nbp_wgrad_group): all the 128-multiple weight gradients of a
// U-Net level's NAFBlocks (conv5's U, conv4, conv3's U with the per-image SCA scale, conv1) are queued while the
// level's backward runs and launched together, with the M-splits chosen for the whole group (few or no splits when
// the group alone fills the chip: the slabs shrink and so do their reductions).
constexpr int WG_MAX = 24;
struct WGroup {
  WgradP p[WG_MAX];
  int gx[WG_MAX], gy[WG_MAX], start[WG_MAX + 1];
  unsigned char xscale[WG_MAX];
  int n;
};

// NT = 64 (2 WNW + 4): the loader / consumer split (wgrad_wide_tile_glds LW).  WNW = 4 (256-column tiles): plain
// problems only (the per-image scale's fold registers do not fit beside 12 waves)
template <typename H, int NS, int NT = 256, int WNW = 2>
__global__ __launch_bounds__(NT) void wgrad_bf16_wide_group(WGroup g) {
  constexpr int SM = NS == 0 ? WIDE_LDS * (int)sizeof(H) : wide_glds_lds_bytes<(NS == 0 ? 2 : NS), WNW>();
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM];
  // consecutive tiles (the N tiles of one K tile and split, which share the X rows) on one XCD and its L2: middle-level
  // group 201.7 -> 188.3 us, 32 x 32 level 183.0 -> 166.6 us (profiles/r04/ab_wgrad_group_variants.txt)
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  int i = 0;
  while (i + 1 < g.n && g.start[i + 1] <= b) ++i;
  const int l = b - g.start[i];
  const int gx = g.gx[i], gy = g.gy[i];
  const int bx = l % gx, by = (l / gx) % gy, bz = l / (gx * gy);
  if constexpr (NS == 0) {
    H* lds = reinterpret_cast<H*>(smem);
    if (g.xscale[i]) wgrad_wide_tile<AM_SCALE, H>(g.p[i], bx, by, bz, lds);
    else wgrad_wide_tile<AM_PLAIN, H>(g.p[i], bx, by, bz, lds);
  } else {
    constexpr bool LW = NT == 64 * (2 * WNW + 4);
    if constexpr (WNW == 4) {
      wgrad_wide_tile_glds<AM_PLAIN, H, NS, 4, LW>(g.p[i], bx, by, bz, smem);
    } else {
      if (g.xscale[i]) wgrad_wide_tile_glds<AM_SCALE, H, NS, 2, LW>(g.p[i], bx, by, bz, smem);
      else wgrad_wide_tile_glds<AM_PLAIN, H, NS, 2, LW>(g.p[i], bx, by, bz, smem);
    }
  }
}

// Column sums of a [S][L] fp32 slab.  A lane sums VEC adjacent columns (float4 loads when VEC = 4) over the rows
// s = ty (mod TY) with 8 independent accumulators (8 loads in flight), combined in a fixed tree; the TY row-lanes of
// a column are then combined in fixed order through LDS.  Bitwise reproducible.
template <int VEC>
__device__ __forceinline__ void slab_col_partial(const float* __restrict__ base, int S, long L, long col, int ty,
                                                 int TY, float* out) {
  typedef float vf __attribute__((ext_vector_type(VEC)));
  vf a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = (vf)0.f;
  int s = ty;
  for (; s + 7 * TY < S; s += 8 * TY) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += *reinterpret_cast<const vf*>(base + (long)(s + u * TY) * L + col);
  }
  for (int u = 0; s < S; s += TY, ++u) a[u & 7] += *reinterpret_cast<const vf*>(base + (long)s * L + col);
  const vf t = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#pragma unroll
  for (int v = 0; v < VEC; ++v) out[v] = t[v];
}

// out[b][i] = scale * sum_{s < S} slab[b][s][i] (exported batched form; 4 row-lanes x 64 columns per block)
__global__ __launch_bounds__(256) void reduce_slab_kernel(const float* __restrict__ slab, int S, long L, float scale,
                                                          float* __restrict__ out) {
  __shared__ float red[4][65];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const long col = (long)blockIdx.x * 64 + tx;
  float v = 0.f;
  if (col < L) slab_col_partial<1>(slab + (long)blockIdx.y * S * L, S, L, col, ty, 4, &v);
  red[ty][tx] = v;
  __syncthreads();
  if (ty == 0 && col < L) out[(long)blockIdx.y * L + col] = (((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx]) * scale;
}

void launch_reduce(const float* slab, int batch, int S, long L, float scale, float* out, hipStream_t st) {
  reduce_slab_kernel<<<dim3(cdiv(L, 64), batch), 256, 0, st>>>(slab, S, L, scale, out);
}

// ---------------------------------------------------------------- deferred gradient reductions
// While deferral is on for a stream, gradient-slab reductions issued on it are queued and later executed by ONE
// launch of reduce_multi_kernel (descriptors passed by value in the kernel arguments); with deferral off a single
// descriptor is launched at once through the same kernel (bitwise identical results).  Per descriptor: TY row-lanes
// (each summing <= 32 rows) x (256 / TY) lanes of VEC columns per block.  The queue is thread-local; callers keep
// the slabs alive until the flush.
struct RDesc {
  const float* slab;
  float* out;
  long L;
  int S, ty, vec, blk0;
};
constexpr int RB_MAX = 48;
// Layer-scale gradient rows reduced straight from the U / V weight-gradient slabs in the same launch (one block per
// row k: U[k][:] = sum_s slabU[s][k][:], V[k] = sum_s slabV[s][k], then the layer_scale_grad_kernel post-op below),
// so a stage flush is one launch and U / V are never written.
struct LDesc {
  const float *slabU, *slabV, *W, *b, *scale;
  float *dW, *db, *dscale;
  int SU, SV, N, K, blk0;
};
constexpr int LB_MAX = 8;
struct RBatch {
  RDesc d[RB_MAX];
  int n;
  LDesc l[LB_MAX];
  int nl, lblk0;
};

RDesc make_rdesc(const float* slab, int S, long L, float* out) {
  int ty = 1;
  while (ty < 64 && (long)ty * 32 < S) ty <<= 1;
  const bool v4 = L % 4 == 0 && (reinterpret_cast<uintptr_t>(slab) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  return RDesc{slab, out, L, S, ty, v4 ? 4 : 1, 0};
}
long rdesc_blocks(const RDesc& d) { return cdiv(d.L, (long)(256 / d.ty) * d.vec); }

__device__ void layer_scale_row_d(const LDesc& d, int lb, float* red) {
  const int row = lb - d.blk0, K = d.K, N = d.N;
  int txq = 1;
  while (txq * 4 < K) txq <<= 1;  // column lanes (4 columns each), a power of two <= 256 (K <= 1024)
  const int TY = 256 / txq, tx = threadIdx.x % txq, ty = threadIdx.x / txq;
  const int col = tx * 4;
  float u[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < K) slab_col_partial<4>(d.slabU + (long)row * K, d.SU, (long)N * K, col, ty, TY, u);
#pragma unroll
  for (int e = 0; e < 4; ++e) red[threadIdx.x * 4 + e] = u[e];
  // V[row]: 256 strided partial sums, folded in fixed order below
  float v = 0.f;
  for (int s2 = threadIdx.x; s2 < d.SV; s2 += 256) v += d.slabV[(long)s2 * N + row];
  __syncthreads();
  const float sc = d.scale[row];
  float dot = 0.f;
  if (ty == 0 && col < K) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int y = 0; y < TY; ++y)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] += red[(y * txq + tx) * 4 + e];
    const float4 w = ld4(d.W + (long)row * K + col);
    dot = fmaf(w.x, t[0], fmaf(w.y, t[1], fmaf(w.z, t[2], w.w * t[3])));
    st4(d.dW + (long)row * K + col, make_float4(sc * t[0], sc * t[1], sc * t[2], sc * t[3]));
  }
  __syncthreads();
  red[threadIdx.x] = v;
  red[256 + threadIdx.x] = dot;
  __syncthreads();
  if (threadIdx.x == 0) {
    float vs = 0.f, ds = 0.f;
    for (int i = 0; i < 256; ++i) vs += red[i];
    for (int i = 0; i < txq; ++i) ds += red[256 + i];
    d.dscale[row] = ds + d.b[row] * vs;
    d.db[row] = sc * vs;
  }
}

__device__ void layer_scale_row(const RBatch& rb, int lb, float* red) {
  int j = 0;
  while (j + 1 < rb.nl && rb.l[j + 1].blk0 <= lb) ++j;
  layer_scale_row_d(rb.l[j], lb, red);
}

__device__ void reduce_desc_block(const RDesc& d, int bid, float* red);

__global__ __launch_bounds__(256) void reduce_multi_kernel(RBatch rb) {
  __shared__ float red[256 * 4];
  const int bid = blockIdx.x;
  if (bid >= rb.lblk0) {
    layer_scale_row(rb, bid - rb.lblk0, red);
    return;
  }
  int k = 0;
  while (k + 1 < rb.n && rb.d[k + 1].blk0 <= bid) ++k;
  reduce_desc_block(rb.d[k], bid, red);
}

// one flush as ONE launch: the descriptors in a device table (written by reduce_desc_write from by-value batches, so
// a captured graph replays them), each block's found by binary search on blk0; the same per-descriptor code
__global__ __launch_bounds__(256) void reduce_table_kernel(const RDesc* __restrict__ dd, int n, const LDesc* __restrict__ dl,
                                                           int nl, int lblk0) {
  __shared__ float red[256 * 4];
  const int bid = blockIdx.x;
  if (bid >= lblk0) {
    const int lb = bid - lblk0;
    int lo = 0, hi = nl - 1;  // the last descriptor with blk0 <= lb
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (dl[mid].blk0 <= lb) lo = mid;
      else hi = mid - 1;
    }
    const LDesc d = dl[lo];
    layer_scale_row_d(d, lb, red);
    return;
  }
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (dd[mid].blk0 <= bid) lo = mid;
    else hi = mid - 1;
  }
  const RDesc d = dd[lo];
  reduce_desc_block(d, bid, red);
}

__global__ __launch_bounds__(64) void reduce_desc_write(RBatch rb, RDesc* __restrict__ dd, LDesc* __restrict__ dl) {
  const int t = threadIdx.x;
  if (t < rb.n) dd[t] = rb.d[t];
  if (t < rb.nl) dl[t] = rb.l[t];
}

__device__ void reduce_desc_block(const RDesc& d, int bid, float* red) {
  const int TY = d.ty, TXQ = 256 / TY, VEC = d.vec;
  const int tx = threadIdx.x % TXQ, ty = threadIdx.x / TXQ;
  const long col = ((long)(bid - d.blk0) * TXQ + tx) * VEC;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < d.L) {
    if (VEC == 4) slab_col_partial<4>(d.slab, d.S, d.L, col, ty, TY, v);
    else slab_col_partial<1>(d.slab, d.S, d.L, col, ty, TY, v);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[(ty * TXQ + tx) * 4 + e] = v[e];
  __syncthreads();
  if (ty == 0 && col < d.L) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < TY; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] += red[(j * TXQ + tx) * 4 + e];
    if (VEC == 4) st4(d.out + col, make_float4(t[0], t[1], t[2], t[3]));
    else d.out[col] = t[0];
  }
}

// Measurement records of the last call of this thread (nbp_last_call_stats; bench.py's per-launch roofline accounting):
// [0] = slabs + layer-scale rows reduced, [1] = slab bytes read, [2] = bytes written, [3] = reduce_multi_kernel launches
thread_local double g_stats_flush[4];
// the last nbp_wgrad_f32 call: [0] = queued into the open group (1) or launched (0), [1] = M-splits, [2] = fp32 slab
// bytes written (at the standalone splits), [3] = FLOPs 2 M N K
thread_local double g_stats_wgrad[4];
// the last group launch: [0] = problems, [1] = FLOPs, [2] = operand bytes read once, [3] = fp32 dW / db bytes,
// [4] = fp32 slab bytes written at the group's M-splits, [5] = kernel launches
thread_local double g_stats_group[6];

// the flush's device descriptor table, per device: grown outside graph capture only, never freed (a captured graph
// keeps addressing the table it was captured with); NBP_REDUCE_TABLE=0: the batched launches
bool reduce_table(hipStream_t st, int nd, int nl, RDesc** dd, LDesc** dl) {
  static const bool on = [] {
    const char* e = getenv("NBP_REDUCE_TABLE");
    return !e || atoi(e) != 0;
  }();
  struct Tab { void* p = nullptr; int cd = 0, cl = 0; };
  static Tab tabs[64];
  int dev = 0;
  if (!on || hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
  Tab& t = tabs[dev];
  if (t.cd < nd || t.cl < nl) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    const int cd = nd > 4096 ? nd : 4096, cl = nl > 512 ? nl : 512;
    void* q = nullptr;
    if (hipMalloc(&q, (size_t)cd * sizeof(RDesc) + (size_t)cl * sizeof(LDesc)) != hipSuccess) return false;
    t.p = q;  // (the previous table stays allocated)
    t.cd = cd;
    t.cl = cl;
  }
  *dd = reinterpret_cast<RDesc*>(t.p);
  *dl = reinterpret_cast<LDesc*>(reinterpret_cast<char*>(t.p) + (size_t)t.cd * sizeof(RDesc));
  return true;
}

void launch_multi(const std::vector<RDesc>& ds, hipStream_t st, const std::vector<LDesc>& ls = {}) {
  static const bool log = getenv("NBP_REDUCE_LOG") != nullptr;  // diagnostic: the flush's descriptors to stderr
  if (log) {
    long bytes = 0;
    for (const RDesc& d : ds) bytes += (long)d.S * d.L * 4;
    for (const LDesc& l : ls) bytes += (long)l.SU * l.N * l.K * 4 + (long)l.SV * l.N * 4;
    fprintf(stderr, "[reduce] flush: %zu slabs + %zu layer-scale, %.2f MB:", ds.size(), ls.size(), bytes / 1e6);
    for (const RDesc& d : ds) fprintf(stderr, " %dx%ld", d.S, d.L);
    for (const LDesc& l : ls) fprintf(stderr, " U%dx%dx%d/V%d", l.SU, l.N, l.K, l.SV);
    fprintf(stderr, "\n");
  }
  {  // measurement record of this flush (nbp_last_call_stats(1, ...))
    double rd = 0, wr = 0;
    for (const RDesc& d : ds) rd += (double)d.S * d.L * 4, wr += (double)d.L * 4;
    for (const LDesc& l : ls) rd += (double)l.SU * l.N * l.K * 4 + (double)l.SV * l.N * 4, wr += (double)l.N * (l.K + 2) * 4;
    g_stats_flush[0] += (double)(ds.size() + ls.size());
    g_stats_flush[1] += rd;
    g_stats_flush[2] += wr;
  }
  RDesc* dd = nullptr;
  LDesc* dl = nullptr;
  if ((ds.size() > (size_t)RB_MAX || ls.size() > (size_t)LB_MAX) &&
      reduce_table(st, (int)ds.size(), (int)ls.size(), &dd, &dl)) {
    // one launch: the descriptors written in by-value batches, blk0 over the whole flush
    long blocks = 0;
    int lblocks = 0;
    double by = 0;
    size_t i = 0, j = 0;
    while (i < ds.size() || j < ls.size()) {
      RBatch rb;
      rb.n = rb.nl = 0;
      const size_t i0 = i, j0 = j;
      for (; i < ds.size() && rb.n < RB_MAX; ++i) {
        RDesc d = ds[i];
        d.blk0 = (int)blocks;
        blocks += rdesc_blocks(d);
        by += (double)d.S * d.L * 4 + (double)d.L * 4;
        rb.d[rb.n++] = d;
      }
      for (; j < ls.size() && rb.nl < LB_MAX; ++j) {
        LDesc d = ls[j];
        d.blk0 = lblocks;
        lblocks += d.N;
        by += (double)d.SU * d.N * d.K * 4 + (double)d.SV * d.N * 4 + (double)d.N * (d.K + 2) * 4;
        rb.l[rb.nl++] = d;
      }
      reduce_desc_write<<<1, 64, 0, st>>>(rb, dd + i0, dl + j0);
    }
    lt_begin(st);
    reduce_table_kernel<<<(unsigned)(blocks + lblocks), 256, 0, st>>>(dd, (int)ds.size(), dl, (int)ls.size(),
                                                                       (int)blocks);
    lt_end(st, "reduce_table_kernel", 0.0, by);
    g_stats_flush[3] += 1;
    return;
  }
  size_t i = 0, j = 0;
  while (i < ds.size() || j < ls.size()) {
    RBatch rb;
    rb.n = rb.nl = 0;
    long blocks = 0;
    for (; i < ds.size() && rb.n < RB_MAX; ++i) {
      RDesc d = ds[i];
      d.blk0 = (int)blocks;
      blocks += rdesc_blocks(d);
      rb.d[rb.n++] = d;
    }
    rb.lblk0 = (int)blocks;
    int lblocks = 0;
    for (; j < ls.size() && rb.nl < LB_MAX; ++j) {
      LDesc d = ls[j];
      d.blk0 = lblocks;
      lblocks += d.N;
      rb.l[rb.nl++] = d;
    }
    double by = 0;  // this launch's slabs read once + outputs written once
    for (int k = 0; k < rb.n; ++k) by += (double)rb.d[k].S * rb.d[k].L * 4 + (double)rb.d[k].L * 4;
    for (int k = 0; k < rb.nl; ++k)
      by += (double)rb.l[k].SU * rb.l[k].N * rb.l[k].K * 4 + (double)rb.l[k].SV * rb.l[k].N * 4 +
            (double)rb.l[k].N * (rb.l[k].K + 2) * 4;
    lt_begin(st);
    reduce_multi_kernel<<<(unsigned)(blocks + lblocks), 256, 0, st>>>(rb);
    lt_end(st, "reduce_multi_kernel", 0.0, by);
    g_stats_flush[3] += 1;
  }
}

// Layer-scale gradient post-op (NAFBlock y = x + beta * conv(h), NAFNet_arch.py:72,80), from U = dOut^T h and
// V = colsum dOut of the UNSCALED output gradient:  dW = s (.) U (rows), db = s (.) V,
// ds[k] = sum_n W[k][n] U[k][n] + b[k] V[k]   (= sum_m dOut[m][k] * conv(h)[m][k]).
// One wave per row k; descriptors by value like RBatch; fixed-order wave sum (deterministic).
struct PDesc {
  const float *U, *V, *W, *b, *scale;
  float *dW, *db, *dscale;
  int N, K, blk0, pad;
};
constexpr int PB_MAX = 24;
struct PBatch {
  PDesc d[PB_MAX];
  int n;
};

__global__ __launch_bounds__(64) void layer_scale_grad_kernel(PBatch pb) {
  const int bid = blockIdx.x;
  int k = 0;
  while (k + 1 < pb.n && pb.d[k + 1].blk0 <= bid) ++k;
  const PDesc& d = pb.d[k];
  const int row = bid - d.blk0, K = d.K, lane = threadIdx.x;
  const float sc = d.scale[row];
  const float* u = d.U + (long)row * K;
  const float* w = d.W + (long)row * K;
  float acc = 0.f;
  for (int i = lane; i < K; i += 64) {
    const float ui = u[i];
    acc = fmaf(w[i], ui, acc);
    d.dW[(long)row * K + i] = sc * ui;
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    const float v = d.V[row];
    d.dscale[row] = acc + d.b[row] * v;
    d.db[row] = sc * v;
  }
}

void launch_post(const std::vector<PDesc>& ops, hipStream_t st) {
  size_t i = 0;
  while (i < ops.size()) {
    PBatch pb;
    pb.n = 0;
    int blocks = 0;
    for (; i < ops.size() && pb.n < PB_MAX; ++i) {
      PDesc d = ops[i];
      d.blk0 = blocks;
      blocks += d.N;
      pb.d[pb.n++] = d;
    }
    double by = 0;  // U, V, W, b, scale read; dW, db, dscale written
    for (int k = 0; k < pb.n; ++k) by += (double)pb.d[k].N * (2.0 * pb.d[k].K + 4) * 4 + (double)pb.d[k].N * 2 * 4;
    lt_begin(st);
    layer_scale_grad_kernel<<<blocks, 64, 0, st>>>(pb);
    lt_end(st, "layer_scale_grad_kernel", 0.0, by);
  }
}

thread_local std::vector<RDesc> g_pending;
thread_local std::vector<PDesc> g_post;
thread_local bool g_defer = false;
thread_local hipStream_t g_defer_stream = nullptr;

// scale-1 reduction of a gradient slab: queued while deferral is on (from any stream of this thread: the caller orders
// the flush after every stream that produced a queued slab), launched otherwise
void grad_reduce(const float* slab, int S, long L, float* out, hipStream_t st) {
  if (g_defer) {
    g_pending.push_back(make_rdesc(slab, S, L, out));
    return;
  }
  launch_multi(std::vector<RDesc>{make_rdesc(slab, S, L, out)}, st);
}

void flush_pending() {
  for (double& v : g_stats_flush) v = 0;
  // a post-op whose U and V are both reductions of this flush becomes a layer-scale row descriptor of the same launch
  std::vector<LDesc> ls;
  std::vector<PDesc> post;
  for (const PDesc& p : g_post) {
    int iu = -1, iv = -1;
    for (int i = 0; i < (int)g_pending.size(); ++i) {
      if (g_pending[i].out == p.U) iu = i;
      if (g_pending[i].out == p.V) iv = i;
    }
    const bool ok = iu >= 0 && iv >= 0 && p.K % 4 == 0 && p.K <= 1024 &&
                    g_pending[iu].L == (long)p.N * p.K && g_pending[iv].L == p.N &&
                    (reinterpret_cast<uintptr_t>(g_pending[iu].slab) & 15) == 0 &&
                    (reinterpret_cast<uintptr_t>(p.W) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.dW) & 15) == 0;
    if (!ok) {
      post.push_back(p);
      continue;
    }
    ls.push_back(LDesc{g_pending[iu].slab, g_pending[iv].slab, p.W, p.b, p.scale, p.dW, p.db, p.dscale,
                       g_pending[iu].S, g_pending[iv].S, p.N, p.K, 0});
    const int hi = iu > iv ? iu : iv, lo = iu > iv ? iv : iu;
    g_pending.erase(g_pending.begin() + hi);
    g_pending.erase(g_pending.begin() + lo);
  }
  launch_multi(g_pending, g_defer_stream, ls);
  g_pending.clear();
  if (!post.empty()) g_stats_flush[3] += 1;
  launch_post(post, g_defer_stream);  // post-ops read reduction outputs: after every reduction of the flush
  g_post.clear();
}

template <int BM, int BN, bool B_NK, int AMODE, int CMODE>
void launch_gemm(const GemmP& p, hipStream_t st) {
  dim3 grid(cdiv(p.M, BM), cdiv(p.N, BN));
  gemm_f32_kernel<BM, BN, B_NK, AMODE, CMODE><<<grid, 256, 0, st>>>(p);
}

template <bool B_NK, int AMODE, int CMODE>
void dispatch_tiles(const GemmP& p, hipStream_t st) {
  const bool bn128 = p.N >= 128;
  const long tiles128 = (long)cdiv(p.M, 128) * cdiv(p.N, bn128 ? 128 : 64);
  const bool bm128 = tiles128 >= 1024;
  if (bm128 && bn128) launch_gemm<128, 128, B_NK, AMODE, CMODE>(p, st);
  else if (bm128) launch_gemm<128, 64, B_NK, AMODE, CMODE>(p, st);
  else if (bn128) launch_gemm<64, 128, B_NK, AMODE, CMODE>(p, st);
  else launch_gemm<64, 64, B_NK, AMODE, CMODE>(p, st);
}

bool wide_wgrad(int N, int K) { return N % 128 == 0 && K % 128 == 0; }

// split-M count: enough blocks to fill the chip (~1024), >= 256 rows per split, and fp32 slab bytes
// (S * N * K * 4, written once and read once by the reduction) no larger than the operand bytes M * (N + K) * 2.
int wgrad_splits(int M, int N, int K) {
  if (wide_wgrad(N, K)) {  // 128 x 128 tiles: ~256 workgroups, >= 256 rows per split
    constexpr long target = 256;
    const long tiles = (long)(N / 128) * (K / 128);
    long s = (target + tiles - 1) / tiles;
    const long maxs = M / 256 > 1 ? M / 256 : 1;
    if (s > maxs) s = maxs;
    return (int)(s > 1024 ? 1024 : s);
  }
  // ~1024 blocks: at levels 0 / 1 the fp32 slabs of ~2048 blocks (up to 32 MB for a 32 KB gradient, 106 MB per
  // stage flush at level 1: NBP_REDUCE_LOG) cost more to write and reduce than the extra blocks gain (A/B: 2048 ->
  // 1024 +0.5 %, 512 +0.2 %, 256 -3.5 %)
  const long tiles = (long)cdiv(N, 64) * cdiv(K, 64);
  long s = (1024 + tiles - 1) / tiles;
  const long maxs = cdiv(M, 256);  // keep >= 256 rows per split
  if (s > maxs) s = maxs;
  const long slab_cap = (long)M * (N + K) / (2L * N * K);
  if (s > slab_cap) s = slab_cap;
  if (s < 1) s = 1;
  if (s > 1024) s = 1024;  // (a cap of 512 / 256 splits: -0.4 / -2.9 %)
  return (int)s;
}

}  // namespace

extern "C" {

int nbp_gemm_f32(const float* A, long lda, int a_mode, const float* a_scale, int rows_per_img, const float* B,
                 long ldb, int b_nk, float* C, long ldc, int c_mode, int M, int N, int K, int gh, int gw, int cs,
                 const float* bias, const float* R, const float* rscale, float* pre, nbp_stream_t s) {
  NBP_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0, "nbp_gemm_f32: null pointer or empty shape");
  NBP_REQUIRE(K % 4 == 0 && N % 4 == 0, "nbp_gemm_f32: K and N must be multiples of 4 (K=%d N=%d)", K, N);
  NBP_REQUIRE(a_mode >= 0 && a_mode <= 2 && c_mode >= 0 && c_mode <= 1, "nbp_gemm_f32: mode");
  NBP_REQUIRE(a_mode != AM_SCALE || (a_scale && rows_per_img > 0), "nbp_gemm_f32: a_scale");
  NBP_REQUIRE((a_mode != AM_S2D && c_mode != CM_D2S) || (gh > 0 && gw > 0 && cs > 0 && cs % 4 == 0),
              "nbp_gemm_f32: s2d geometry");
  NBP_REQUIRE(a_mode != AM_S2D || K == 4 * cs, "nbp_gemm_f32: S2D needs K == 4*cs");
  NBP_REQUIRE(c_mode != CM_D2S || N == 4 * cs, "nbp_gemm_f32: D2S needs N == 4*cs");
  NBP_REQUIRE(a_mode == AM_S2D || lda % 4 == 0, "nbp_gemm_f32: lda alignment");
  GemmP p{A, lda, a_scale, rows_per_img, B, ldb, C, ldc, M, N, K, gh, gw, cs, bias, R, rscale, pre,
          0, 0, 0, 0, 0, 0, 0};
  hipStream_t st = S(s);
  if (b_nk) {
    if (a_mode == AM_PLAIN && c_mode == CM_PLAIN) dispatch_tiles<true, AM_PLAIN, CM_PLAIN>(p, st);
    else if (a_mode == AM_SCALE && c_mode == CM_PLAIN) dispatch_tiles<true, AM_SCALE, CM_PLAIN>(p, st);
    else if (a_mode == AM_S2D && c_mode == CM_PLAIN) dispatch_tiles<true, AM_S2D, CM_PLAIN>(p, st);
    else if (a_mode == AM_PLAIN && c_mode == CM_D2S) dispatch_tiles<true, AM_PLAIN, CM_D2S>(p, st);
    else { set_error("nbp_gemm_f32: unsupported NK mode combination"); return NBP_ERR_ARG; }
  } else {
    if (a_mode == AM_PLAIN && c_mode == CM_PLAIN) dispatch_tiles<false, AM_PLAIN, CM_PLAIN>(p, st);
    else if (a_mode == AM_PLAIN && c_mode == CM_D2S) dispatch_tiles<false, AM_PLAIN, CM_D2S>(p, st);
    else if (a_mode == AM_S2D && c_mode == CM_PLAIN) dispatch_tiles<false, AM_S2D, CM_PLAIN>(p, st);
    else if (a_mode == AM_SCALE && c_mode == CM_PLAIN) dispatch_tiles<false, AM_SCALE, CM_PLAIN>(p, st);
    else { set_error("nbp_gemm_f32: unsupported KN mode combination"); return NBP_ERR_ARG; }
  }
  return check_launch("gemm_f32");
}

}  // extern "C"

namespace nbp {
// fp32 implicit-GEMM convolution (the parity mode of the VGG / LPIPS trunks: the reference's PerceptualLoss runs its
// conv stack in fp32, NewBP_model/losses.py:63-69): y[b][oi][oj][n] = epi(sum_{ki,kj,c} x[b][oi*s+ki-p][oj*s+kj-p][c]
// * w[n][ki*KW+kj][c] (+ bias[n])) on v_mfma_f32_32x32x2_f32 (exact products, fp32 accumulation).
// mode 0 bias + ReLU, 1 bias (or none), 2 ReLU-mask by R (no bias).  Cin, Cout multiples of 4.
int conv_f32(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int KH, int KW, int stride, int pad,
             const float* bias, int mode, const float* R, float* y, hipStream_t st) {
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  NBP_REQUIRE(Ho > 0 && Wo > 0 && Cin % 4 == 0 && Cout % 4 == 0, "conv_f32: shape");
  const long M = (long)B * Ho * Wo;
  NBP_REQUIRE(M < (1L << 31), "conv_f32: too many pixels");
  const int K = KH * KW * Cin;
  GemmP p{x, 0, nullptr, 1, w, (long)K, y, Cout, (int)M, Cout, K, Ho, Wo, 0, mode == 2 ? nullptr : bias,
          mode == 2 ? R : nullptr, nullptr, nullptr, H, W, Cin, KH, KW, stride, pad};
  if (mode == 0) dispatch_tiles<true, AM_CONV, CM_RELU>(p, st);
  else if (mode == 2) dispatch_tiles<true, AM_CONV, CM_MASK>(p, st);
  else dispatch_tiles<true, AM_CONV, CM_PLAIN>(p, st);
  return check_launch("conv_f32");
}
}  // namespace nbp

extern "C" {

size_t nbp_wgrad_workspace_floats(int M, int N, int K) {
  const int S_ = std::max(wgrad_splits(M, N, K), wgrad_full_splits(M));
  return (size_t)S_ * N * K + (size_t)S_ * N;
}

thread_local bool g_wgroup = false;
thread_local std::vector<WgradP> g_wqueue;
thread_local int g_wqueue_dtype = 1;  // the 16-bit type of the queued problems (one per group)

// M-splits of a group launch kind with `tiles` output tiles (one resident workgroup per CU): the split count S
// minimising rounds x (1 / S + per-workgroup overhead) + slab cost, rounds = ceil(tiles S / CUs) -- i.e. the fewest
// splits that still fill the last round (middle level: the 256-column tiles unsplit in one round, the 128-column
// scale tiles in two halves).
int wgroup_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}
long wgroup_splits(long tiles, long cap) {
  const long cus = wgroup_cus();
  long best = 1;
  double best_c = 1e30;
  for (long sp = 1; sp <= cap && sp <= 64; ++sp) {
    const double c = (double)((tiles * sp + cus - 1) / cus) * (1.0 / sp + 0.07) + 0.02 * sp;
    if (c < best_c - 1e-9) best_c = c, best = sp;
  }
  return best;
}

// Row-stage height of the narrow (N or K <= 64) weight-gradient tiles: 64 (measured +0.3 % at cfg2 over 32-row
// stages, bitwise equal, profiles/r02_v6/ab_wgrad_rm.txt; 128-row and double-buffered 64-row stages were measured
// slower).  32-row stages remain where a per-image scale block is not a multiple of 64 rows.

// NBP_WGRAD_GLDS: LDS-DMA ring depth of the wide weight-gradient tiles (2 or 3; 0 = register-staged tiles), read per
// launch (A/B measurement; tests compare the paths in one process)
int wgrad_glds_depth() {  // 3: +1.6 % step over the register-staged tiles, +0.5 % over depth 2 (A/B)
  // 43 / 44 (round 4): the loader / consumer split (8 waves) with a 3- / 4-deep ring, in the grouped launch only;
  // 83 (default): 43 plus the 256-column tiles where they fill one round (wgroup_launch)
  const char* e = getenv("NBP_WGRAD_GLDS");
  const int v = e ? atoi(e) : 83;
  return (v >= 2 && v <= 4) || v == 43 || v == 44 || v == 83 || v == 84 ? v : 0;
}

// Splits per launch kind of the group (wgroup_splits): each problem keeps at most its standalone split count (its
// workspace) and at least 256 rows per split.  The reductions queued for the
// problems' slabs are re-pointed at the chosen split counts.
void wgroup_launch_chunk(hipStream_t st, int ns, int q0, int q1) {
  // 83 / 84: plain problems with N % 256 == 0 on 256 x 128 tiles (8 compute + 4 loader waves), the rest as 43 / 44
  // -- where those tiles fill the chip in ONE unsplit round (the middle level: 240 tiles); elsewhere the split 256-
  // column tiles measured slower than the 128-column ones (32 x 32 level 119 -> 130 us, 64 x 64 119 -> 240 us)
  bool w4 = ns == 83 || ns == 84;
  auto plain256 = [](const WgradP& p) { return p.x_scale == nullptr && p.N % 256 == 0; };
  if (w4) {
    long t4 = 0;
    for (int q = q0; q < q1; ++q)
      if (plain256(g_wqueue[q])) t4 += (long)(g_wqueue[q].N / 256) * (g_wqueue[q].K / 128);
    w4 = t4 > wgroup_cus() / 2 && t4 <= wgroup_cus();
  }
  auto wide4 = [&](const WgradP& p) { return w4 && plain256(p); };
  long tiles[2] = {0, 0};  // per launch kind: 128- / 256-column tiles
  for (int q = q0; q < q1; ++q) {
    const WgradP& p = g_wqueue[q];
    tiles[wide4(p)] += (long)(p.N / (wide4(p) ? 256 : 128)) * (p.K / 128);
  }
  long want[2] = {1, 1};  // kind 1 unsplit; the 128-column tiles packed by wgroup_splits
  if (tiles[0]) want[0] = wgroup_splits(tiles[0], 64);
  if (const char* e = getenv("NBP_WGROUP_SPLITS"))  // (test hook: equal splits for the bitwise variant comparison)
    if (atoi(e) > 0) want[0] = want[1] = atoi(e);
  for (int q = q0; q < q1; ++q) {
    WgradP& p = g_wqueue[q];
    const long s_max = cdiv(p.M, p.chunk);  // (the problem's workspace holds its standalone split count)
    long s = want[wide4(p)] < s_max ? want[wide4(p)] : s_max;
    const long rows_cap = p.M / 256 > 1 ? p.M / 256 : 1;
    if (s > rows_cap) s = rows_cap;
    if (s < 1) s = 1;
    p.chunk = cdiv(cdiv(p.M, (int)s), 64) * 64;
    const int S_ = cdiv(p.M, p.chunk);
    const int es = g_wqueue_dtype != 0 ? 2 : 4;
    bool direct = false;
    if (S_ == 1) {
      // one split: the tile writes the weight (and bias) gradient itself and its queued reductions -- copies -- are
      // dropped; not for the layer-scale problems (their U / V are reduced straight from the slabs by the flush)
      auto ls = [](const float* out) {
        for (const PDesc& q : g_post)
          if (q.U == out || q.V == out) return true;
        return false;
      };
      int iw = -1, ib = -1;
      for (int r = 0; r < (int)g_pending.size(); ++r) {
        if (g_pending[r].slab == p.slab) iw = r;
        if (p.slab_b && g_pending[r].slab == p.slab_b) ib = r;
      }
      if (iw >= 0 && !ls(g_pending[iw].out) && (!p.slab_b || (ib >= 0 && !ls(g_pending[ib].out)))) {
        float* ow = g_pending[iw].out;
        float* ob = p.slab_b ? g_pending[ib].out : nullptr;
        if (ib > iw) g_pending.erase(g_pending.begin() + ib);
        g_pending.erase(g_pending.begin() + iw);
        if (ib >= 0 && ib < iw) g_pending.erase(g_pending.begin() + ib);
        p.slab = ow;
        p.slab_b = ob;
        direct = true;
      }
    }
    g_stats_group[0] += 1;
    g_stats_group[1] += 2.0 * p.M * p.N * p.K;
    g_stats_group[2] += (double)p.M * (p.N + p.K) * es;
    g_stats_group[3] += (double)p.N * p.K * 4 + (p.slab_b ? (double)p.N * 4 : 0.0);
    if (!direct) g_stats_group[4] += (double)S_ * p.N * p.K * 4 + (p.slab_b ? (double)S_ * p.N * 4 : 0.0);
    for (RDesc& d : g_pending)
      if (d.slab == p.slab || (p.slab_b && d.slab == p.slab_b)) d.S = S_, d.ty = make_rdesc(d.slab, S_, d.L, d.out).ty;
  }
  for (int kind = 1; kind >= 0; --kind) {
    if (!tiles[kind]) continue;
    const int TNB = kind ? 256 : 128;
    {
      WGroup g;
      g.n = 0;
      int blocks = 0;
      double kfl = 0, kby = 0;  // this launch's algorithmic FLOPs / bytes (operands once, dW / db once)
      for (int q = q0; q < q1; ++q) {
        const WgradP& p = g_wqueue[q];
        if ((int)wide4(p) != kind) continue;
        kfl += 2.0 * p.M * p.N * p.K;
        kby += (double)p.M * (p.N + p.K) * (g_wqueue_dtype != 0 ? 2 : 4) + (double)p.N * p.K * 4 +
               (p.slab_b ? (double)p.N * 4 : 0.0);
        g.p[g.n] = p;
        g.gx[g.n] = p.N / TNB;
        g.gy[g.n] = p.K / 128;
        g.xscale[g.n] = p.x_scale != nullptr;
        g.start[g.n] = blocks;
        blocks += g.gx[g.n] * g.gy[g.n] * cdiv(p.M, p.chunk);
        ++g.n;
      }
      if (!g.n) continue;
      g.start[g.n] = blocks;
      const char* kname = kind ? "wgrad_bf16_wide_group<3,768,4>" : (ns == 44 || ns == 84) ? "wgrad_bf16_wide_group<4,512,2>"
                          : (ns == 43 || ns == 83) ? "wgrad_bf16_wide_group<3,512,2>" : "wgrad_bf16_wide_group<256>";
      lt_begin(st);
      NBP_DISPATCH_H(g_wqueue_dtype, {
        if (kind) {  // (a 4-deep ring of 48-KB stages would not fit in LDS)
          wgrad_bf16_wide_group<H, 3, 768, 4><<<blocks, 768, 0, st>>>(g);
        } else if (ns == 44 || ns == 84) {
          wgrad_bf16_wide_group<H, 4, 512><<<blocks, 512, 0, st>>>(g);
        } else if (ns == 43 || ns == 83) {
          wgrad_bf16_wide_group<H, 3, 512><<<blocks, 512, 0, st>>>(g);
        } else if (ns == 4) {
          wgrad_bf16_wide_group<H, 4><<<blocks, 256, 0, st>>>(g);
        } else if (ns == 3) {
          wgrad_bf16_wide_group<H, 3><<<blocks, 256, 0, st>>>(g);
        } else if (ns == 2) {
          wgrad_bf16_wide_group<H, 2><<<blocks, 256, 0, st>>>(g);
        } else {
          wgrad_bf16_wide_group<H, 0><<<blocks, 256, 0, st>>>(g);
        }
      });
      lt_end(st, kname, kfl, kby);
      g_stats_group[5] += 1;
    }
  }
}
void wgroup_launch(hipStream_t st) {
  for (double& v : g_stats_group) v = 0;
  const int ns = wgrad_glds_depth();
  // the queue (a whole U-Net level) in balanced chunks of <= WG_MAX problems, each chunk one launch per tile kind
  const int nq = (int)g_wqueue.size(), nch = (nq + WG_MAX - 1) / WG_MAX;
  for (int c = 0; c < nch; ++c)
    wgroup_launch_chunk(st, ns, (int)((long)nq * c / nch), (int)((long)nq * (c + 1) / nch));
  g_wqueue.clear();
}


int nbp_wgrad_f32(const void* G, long ldg, int g_mode, const void* X, long ldx, int x_mode, const float* x_scale,
                  int rows_per_img, int M, int N, int K, int gh, int gw, int cs_g, int cs_x, float* dW, float* db,
                  float* ws, size_t ws_floats, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(G && X && dW && ws && M > 0 && N > 0 && K > 0, "nbp_wgrad_f32: null pointer or empty shape");
  NBP_REQUIRE(N % 4 == 0 && K % 4 == 0, "nbp_wgrad_f32: N, K multiples of 4");
  NBP_REQUIRE((g_mode == AM_PLAIN || g_mode == AM_S2D) && x_mode >= 0 && x_mode <= 2, "nbp_wgrad_f32: mode");
  NBP_REQUIRE(g_mode != AM_S2D || (N == 4 * cs_g && gh > 0 && gw > 0), "nbp_wgrad_f32: G s2d geometry");
  NBP_REQUIRE(x_mode != AM_S2D || (K == 4 * cs_x && gh > 0 && gw > 0), "nbp_wgrad_f32: X s2d geometry");
  NBP_REQUIRE(x_mode != AM_SCALE || (x_scale && rows_per_img > 0), "nbp_wgrad_f32: x_scale");
  // the full-width narrow kernel: level-0 / 1 shapes, 16-bit, plain G, plain or per-image-scaled X (64-row stages)
  const bool full = dtype != 0 && wgrad_full_enabled() && g_mode == AM_PLAIN &&
                    (x_mode == AM_PLAIN || (x_mode == AM_SCALE && rows_per_img % 64 == 0 && N * K <= 4096)) &&
                    (N == 32 || N == 64 || N == 128) && (K == 32 || K == 64) && ldg % 8 == 0 && ldx % 8 == 0;
  // ... and the level-0 / 1 down / up conv gradients (one side space-to-depth gathered, 8-channel chunks)
  const bool full_s2d = dtype != 0 && wgrad_full_enabled() &&
                        ((g_mode == AM_PLAIN && x_mode == AM_S2D && N == 64 && K == 128 && ldg % 8 == 0) ||
                         (g_mode == AM_S2D && x_mode == AM_PLAIN && N == 128 && K == 64 && ldx % 8 == 0));
  const int S_ = full || full_s2d ? wgrad_full_splits(M) : wgrad_splits(M, N, K);
  NBP_REQUIRE(ws_floats >= (size_t)S_ * N * K + (size_t)S_ * N, "nbp_wgrad_f32: workspace too small");
  int chunk = cdiv(M, S_);
  chunk = cdiv(chunk, 64) * 64;
  float* slab = ws;
  float* slab_b = db ? ws + (size_t)S_ * N * K : nullptr;
  WgradP p{G, ldg, X, ldx, x_scale, rows_per_img, M, N, K, gh, gw, cs_g, cs_x, slab, slab_b, chunk};
  dim3 grid(cdiv(N, 64), cdiv(K, 64), S_);
  hipStream_t st = S(s);
  bool ok = true;
  g_stats_wgrad[0] = 0;
  g_stats_wgrad[1] = S_;
  g_stats_wgrad[2] = (double)S_ * N * K * 4 + (db ? (double)S_ * N * 4 : 0.0);
  g_stats_wgrad[3] = 2.0 * M * N * K;
  if (dtype != 0) {
    NBP_REQUIRE(N % 8 == 0 && K % 8 == 0 && (g_mode != AM_S2D || cs_g % 8 == 0) && (x_mode != AM_S2D || cs_x % 8 == 0),
                "nbp_wgrad_f32(16-bit): N, K and S2D channel counts must be multiples of 8");
    NBP_REQUIRE((g_mode == AM_S2D || ldg % 8 == 0) && (x_mode == AM_S2D || ldx % 8 == 0),
                "nbp_wgrad_f32(16-bit): leading dimensions must be multiples of 8");
    // every 16-bit kernel below reads G and X by 16-byte vectors from the base pointers (views at odd element offsets
    // would be read from the wrong addresses)
    NBP_REQUIRE((((uintptr_t)G | (uintptr_t)X) & 15) == 0, "nbp_wgrad_f32(16-bit): G and X must be 16-byte aligned");
    const bool wide = wide_wgrad(N, K) && g_mode == AM_PLAIN &&
                      (x_mode == AM_PLAIN || (x_mode == AM_SCALE && rows_per_img % 64 == 0));
    const dim3 wgrid(N / 128, K / 128, S_);
    // grouped only while the slab reductions are deferred (they must run after the queued launch)
    if (wide && g_wgroup && g_defer) {  // nbp_wgrad_group(0, ...) launches
      NBP_REQUIRE(g_wqueue.empty() || g_wqueue_dtype == dtype, "nbp_wgrad_f32: mixed dtypes in one group");
      g_wqueue_dtype = dtype;
      if (x_mode != AM_SCALE) p.x_scale = nullptr;  // the group kernel selects the X mode by x_scale
      g_wqueue.push_back(p);
      g_stats_wgrad[0] = 1;
    } else if (full) {
      NBP_DISPATCH_H(dtype, {
        if (x_mode == AM_PLAIN) launch_wgrad_full<H, AM_PLAIN>(p, S_, st);
        else launch_wgrad_full<H, 3>(p, S_, st);
      });
    } else if (full_s2d) {
      NBP_DISPATCH_H(dtype, launch_wgrad_full_s2d<H>(p, g_mode == AM_S2D, S_, st));
    } else NBP_DISPATCH_H(dtype, {
      const int ns = wgrad_glds_depth() % 10;  // (the loader-split variants are grouped-launch only)
      if (wide && ns == 4 && x_mode == AM_PLAIN) wgrad_bf16_wide_glds<AM_PLAIN, H, 4><<<wgrid, 256, 0, st>>>(p);
      else if (wide && ns == 4) wgrad_bf16_wide_glds<AM_SCALE, H, 4><<<wgrid, 256, 0, st>>>(p);
      else if (wide && ns == 2 && x_mode == AM_PLAIN) wgrad_bf16_wide_glds<AM_PLAIN, H, 2><<<wgrid, 256, 0, st>>>(p);
      else if (wide && ns == 2) wgrad_bf16_wide_glds<AM_SCALE, H, 2><<<wgrid, 256, 0, st>>>(p);
      else if (wide && ns == 3 && x_mode == AM_PLAIN) wgrad_bf16_wide_glds<AM_PLAIN, H, 3><<<wgrid, 256, 0, st>>>(p);
      else if (wide && ns == 3) wgrad_bf16_wide_glds<AM_SCALE, H, 3><<<wgrid, 256, 0, st>>>(p);
      else if (wide && x_mode == AM_PLAIN) wgrad_bf16_wide<AM_PLAIN, H><<<wgrid, 256, 0, st>>>(p);
      else if (wide) wgrad_bf16_wide<AM_SCALE, H><<<wgrid, 256, 0, st>>>(p);
      else if (g_mode == AM_PLAIN && x_mode == AM_PLAIN)
        wgrad_bf16_kernel<AM_PLAIN, AM_PLAIN, H, 64><<<grid, 256, 0, st>>>(p);
      else if (g_mode == AM_PLAIN && x_mode == AM_SCALE && rows_per_img % 64 == 0)
        wgrad_bf16_kernel<AM_PLAIN, 3, H, 64><<<grid, 256, 0, st>>>(p);
      else if (g_mode == AM_PLAIN && x_mode == AM_SCALE && rows_per_img % 32 == 0)
        wgrad_bf16_kernel<AM_PLAIN, 3, H><<<grid, 256, 0, st>>>(p);
      else if (g_mode == AM_PLAIN && x_mode == AM_SCALE) wgrad_bf16_kernel<AM_PLAIN, AM_SCALE, H><<<grid, 256, 0, st>>>(p);
      else if (g_mode == AM_PLAIN && x_mode == AM_S2D) wgrad_bf16_kernel<AM_PLAIN, AM_S2D, H><<<grid, 256, 0, st>>>(p);
      else if (g_mode == AM_S2D && x_mode == AM_PLAIN) wgrad_bf16_kernel<AM_S2D, AM_PLAIN, H><<<grid, 256, 0, st>>>(p);
      else ok = false;
    });
  } else {
    using T = float;
    if (g_mode == AM_PLAIN && x_mode == AM_PLAIN) wgrad_f32_kernel<AM_PLAIN, AM_PLAIN, T><<<grid, 256, 0, st>>>(p);
    else if (g_mode == AM_PLAIN && x_mode == AM_SCALE) wgrad_f32_kernel<AM_PLAIN, AM_SCALE, T><<<grid, 256, 0, st>>>(p);
    else if (g_mode == AM_PLAIN && x_mode == AM_S2D) wgrad_f32_kernel<AM_PLAIN, AM_S2D, T><<<grid, 256, 0, st>>>(p);
    else if (g_mode == AM_S2D && x_mode == AM_PLAIN) wgrad_f32_kernel<AM_S2D, AM_PLAIN, T><<<grid, 256, 0, st>>>(p);
    else ok = false;
  }
  if (!ok) { set_error("nbp_wgrad_f32: unsupported mode combination"); return NBP_ERR_ARG; }
  grad_reduce(slab, S_, (long)N * K, dW, st);
  if (db) grad_reduce(slab_b, S_, N, db, st);
  return check_launch("wgrad_f32");
}

int nbp_reduce_slab(const float* slab, int S_, long L, float* out, nbp_stream_t s) {
  NBP_REQUIRE(slab && out && S_ > 0 && L > 0, "nbp_reduce_slab: bad args");
  grad_reduce(slab, S_, L, out, S(s));
  return check_launch("reduce_slab");
}

int nbp_reduce_slab_batched(const float* slab, int batch, int S_, long L, float scale, float* out, nbp_stream_t s) {
  NBP_REQUIRE(slab && out && batch > 0 && batch <= 65535 && S_ > 0 && L > 0, "nbp_reduce_slab_batched: bad args");
  launch_reduce(slab, batch, S_, L, scale, out, S(s));
  return check_launch("reduce_slab_batched");
}

int nbp_layer_scale_grad(const float* U, const float* V, const float* W, const float* b, const float* scale, float* dW,
                         float* db, float* dscale, int N, int K, nbp_stream_t s) {
  NBP_REQUIRE(U && V && W && b && scale && dW && db && dscale && N > 0 && K > 0, "nbp_layer_scale_grad: bad args");
  PDesc d{U, V, W, b, scale, dW, db, dscale, N, K, 0, 0};
  if (g_defer) {
    g_post.push_back(d);
    return NBP_OK;
  }
  launch_post(std::vector<PDesc>{d}, S(s));
  return check_launch("layer_scale_grad");
}

int nbp_wgrad_group(int begin, nbp_stream_t s) {
  NBP_REQUIRE(begin ? !g_wgroup : g_wgroup, "nbp_wgrad_group: unbalanced begin / end");
  g_wgroup = begin != 0;
  for (double& v : g_stats_group) v = 0;
  if (!begin) wgroup_launch(S(s));
  return check_launch("wgrad_group");
}

int nbp_grad_reduce_defer(nbp_stream_t s) {
  NBP_REQUIRE(!g_defer || (g_pending.empty() && g_post.empty()) || g_defer_stream == S(s),
              "nbp_grad_reduce_defer: reductions pending on another stream");
  g_defer = true;
  g_defer_stream = S(s);
  return NBP_OK;
}

int nbp_last_call_stats(int which, double* out, int n) {
  NBP_REQUIRE(out && n > 0 && which >= 0 && which <= 2, "nbp_last_call_stats: bad args");
  const double* src = which == 0 ? g_stats_wgrad : which == 1 ? g_stats_flush : g_stats_group;
  const int len = which == 2 ? 6 : 4;
  for (int i = 0; i < n; ++i) out[i] = i < len ? src[i] : 0.0;
  return NBP_OK;
}

int nbp_grad_reduce_flush(int stop, nbp_stream_t s) {
  NBP_REQUIRE(!g_defer || g_defer_stream == S(s), "nbp_grad_reduce_flush: deferral is active on another stream");
  for (double& v : g_stats_flush) v = 0;
  if (g_defer) flush_pending();
  if (stop) g_defer = false;
  return check_launch("grad_reduce_flush");
}

}  // extern "C"
