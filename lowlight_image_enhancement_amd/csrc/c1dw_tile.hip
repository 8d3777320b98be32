// Levels 0 / 1 of the NAFBlock spatial branch with the 2C-wide tape kept on chip (VERDICT r4 item 1;
// NAFNet_arch.py:59-68: conv1 (1x1, C -> 2C), conv2 (depthwise 3x3, zero pad 1), SimpleGate, the SCA's pool).
//
// Forward (c1dw_fwd_tile): a workgroup owns a TH x TW pixel tile of one image x one slice of 32 gate channels and their
// 32 SimpleGate partners.  It walks the tile's rows with a 4-slot LDS ring of conv1 output rows (TW + 2 pixels, the
// one-pixel halo, 64 fp32 channels each): per step the MFMA phase forms the next t1 row from the n1 row (32x32x16
// MFMA, the conv1 weight slice as the A operand in registers, the pixels as the B operand loaded in fragment order,
// the n1 rows of the next steps in flight), rounds it to the storage type and widens it into the ring (zeros outside
// the image: the depthwise conv's padding); after one barrier the depthwise phase convolves the middle rows of the ring,
// forms the gate and the pool partials.  t1 and t2 never reach HBM (the backward rebuilds them from n1); per pixel the
// launch reads n1 (C) and writes g (C) instead of conv1's t1 (2C out) + the depthwise pass (2C in, 2C + C out).
//
// Backward (c1dw_bwd_tile): the mirror.  Per output row of dt1 the walk rebuilds t1 on a two-pixel halo (MFMA from n1),
// t2 on a one-pixel halo (depthwise forward), forms dt2 = (dg t2[C:], dg t2[:C]) with dg = dh a + ds / HW (the SCA and
// SimpleGate backward) into a 3-slot dt2 ring, accumulates the depthwise weight / bias gradients of the tile's own dt2
// pixels, and convolves the dt2 ring into dt1 (stored: the conv1 input / weight gradients read it).  Per pixel: dh (C)
// and n1 (C) in, dt1 (2C) out, instead of dh + t2 (2C) + t1 (2C) in and dt1 (2C) out.
//
// Bitwise contract (the GPU tests pin it against the two-launch path): t1 is the skinny conv1's MFMA sequence per
// element (K ascending in steps of 16 on one accumulator, + bias, one rounding), t2 the tiled depthwise kernel's (bias,
// then taps 0..8 by fused multiply-add), the gate the same opaque fp32 product rounded once, dt2 the products of the
// rounded t2 with dg rounded once, dt1 taps 0..8 from zero.  The pool and the depthwise weight gradients are per-tile
// partial sums in an order of their own (equal to the two-launch values up to fp32 summation order).
#include "rowring.h"
#include "sca_bwd.h"

namespace nbp {
namespace {

constexpr int CT_TH = 16;  // tile rows

struct C1TileP {
  const void* n1;     // [B][H][W][C]: the block's norm1 output (conv1 input)
  const void* w1;     // [2C][C] 16-bit forward copy of conv1.weight (rows 0..C-1 gate, C..2C-1 partners)
  const float* b1;    // [2C]
  const float* wdw;   // [2C][9] conv2.weight
  const float* bdw;   // [2C]    conv2.bias
  // forward
  void* t1;           // [M][2C] optional out (null: not kept)
  void* t2;           // [M][2C] optional out (null: not kept)
  void* g;            // [M][C] out
  float* pool;        // [B][tiles][C] out: per-tile pool partial sums of the fp32 gate products
  // backward
  const void* dh;     // [M][C] gradient of the SCA-scaled gate h = g * a
  const float* a;     // [B][C] SCA scale
  const float* ds;    // [B][C] gradient of the pooled mean (d pool sum = ds / HW)
  void* dt1;          // [M][2C] out
  float* slab_w;      // [B * tiles][2C][9] out: per-tile depthwise weight-gradient partials
  float* slab_b;      // [B * tiles][2C]    out: per-tile depthwise bias-gradient partials
  int B, H, W, tiles_x, tiles;
  float inv_hw;
  // backward with the SCA backward folded in (nbp_sca_c1dw_bwd_tile; ds above unused)
  const float* da_slab;  // [B][chunks][C]
  const float* wsca;     // [C][C]
  const float* mean;     // [B][C]
  float* dwsca;          // [C][C] out
  float* dbsca;          // [C] out
  int chunks;
};

// the slice's conv1 weight rows (A operand: n = t * 32 + r, t 0 gate rows slice * 32 + r, 1 partner rows C + ...) in
// registers, and the bias of this lane's output channels t*32 + 8g + 4hh + q
template <typename T, int C>
struct Conv1Rows {
  static constexpr int KS = C / 16;
  vec_t<T, 8> w[2][KS];
  float bias[2][4][4];

  __device__ __forceinline__ void load_weights(const C1TileP& p, int slice, int r, int hh) {
    const T* w1 = reinterpret_cast<const T*>(p.w1);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n = (t == 0 ? 0 : C) + slice * 32 + r;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) w[t][ks] = *reinterpret_cast<const vec_t<T, 8>*>(w1 + (long)n * C + ks * 16 + 8 * hh);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 b = ld4(p.b1 + (t == 0 ? 0 : C) + slice * 32 + 8 * g + 4 * hh);
        bias[t][g][0] = b.x; bias[t][g][1] = b.y; bias[t][g][2] = b.z; bias[t][g][3] = b.w;
      }
    }
  }
};

// the B-operand fragments of one pixel chunk of one image row (zeros outside the image: OOB offsets)
template <typename T, int KS>
__device__ __forceinline__ void load_n1(__amdgpu_buffer_rsrc_t rn, long img, int W, int H, int yy, int gx, bool lane_ok,
                                        int hh, vec_t<T, 8>* f) {
  const bool ok = lane_ok && yy >= 0 && yy < H && gx >= 0 && gx < W;
  const int off = ok ? (int)((img + (long)yy * W + gx) * (KS * 32)) + 16 * hh : OOB;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) f[ks] = bload8<T>(rn, off + 32 * ks);
}

template <typename T, int C, int TW, bool KEEP>
__global__ __launch_bounds__(256, 2) void c1dw_fwd_tile(C1TileP p) {
  constexpr int TH = CT_TH, LW = TW + 2, KS = C / 16, NSL = C / 32;
  constexpr int NCHK = (LW + 31) / 32;  // 32-pixel MFMA chunks per ring row
  constexpr int PXT = TW / 16;          // depthwise pixels per thread (adjacent columns)
  constexpr int ROWF = LW * 64;         // floats per ring row
  constexpr int NR = 4;                 // n1 register-ring slots = the row loop's unroll (3 rows in flight)
  static_assert(NCHK <= 4 && (PXT == 2 || PXT == 4) && TH % NR == 0, "tile geometry");
  __shared__ __attribute__((aligned(16))) float ring[4 * ROWF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, hh = lane >> 5;
  // the slices of one tile, then neighbouring tiles, on one XCD (they share n1 lines: L2 hits)
  const int u = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = u % NSL, tile = (u / NSL) % p.tiles, b = u / (NSL * p.tiles);
  const int y0 = (tile / p.tiles_x) * TH, x0 = (tile % p.tiles_x) * TW;
  const int H = p.H, W = p.W;
  const long img = (long)b * H * W, M = (long)p.B * H * W;
  const __amdgpu_buffer_rsrc_t rn = rsrc(p.n1, M * C * 2), rg = rsrc(p.g, M * C * 2);
  const __amdgpu_buffer_rsrc_t r1 = rsrc(p.t1, KEEP ? M * C * 4 : 0), r2 = rsrc(p.t2, KEEP ? M * C * 4 : 0);
  const bool mfma_wave = wave < NCHK;
  const int gxm = x0 - 1 + wave * 32 + r;  // this lane's MFMA pixel (ring pixel wave * 32 + r)
  const bool lane_ok = wave * 32 + r < LW;
  Conv1Rows<T, C> cw;
  vec_t<T, 8> fq[NR][KS];  // n1 fragments of image row y0 - 1 + k in slot k % NR
  if (mfma_wave) {
    cw.load_weights(p, slice, r, hh);
#pragma unroll
    for (int k = 0; k < NR; ++k) load_n1<T, KS>(rn, img, W, H, y0 - 1 + k, gxm, lane_ok, hh, fq[k]);
  }
  const int q16 = (lane & 7) + 8 * hh, xl = PXT * (4 * wave + ((lane >> 3) & 3));
  const bool gate = hh == 0;
  const int ch = (gate ? 0 : C) + slice * 32 + 4 * (lane & 7);  // this lane's conv channels
  DwQuad dw;
  dw.load(p.wdw, p.bdw, ch);

  // MFMA phase of ring row k (image row y0 - 1 + k) from register slot S = k % NR, which then takes image row k + NR - 1.
  // The epilogue widens the rounded t1 into the ring (zero outside the image); KEEP also stores the tile's own pixels.
  auto mfma_row = [&](auto slot_c, int k) {
    constexpr int S = decltype(slot_c)::value;
    const int yy = y0 - 1 + k;
    const bool valid = yy >= 0 && yy < H && lane_ok && gxm >= 0 && gxm < W;
    floatx16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma32x32x16(cw.w[t][ks], fq[S][ks], acc[t]);
    load_n1<T, KS>(rn, img, W, H, yy + NR, gxm, lane_ok, hh, fq[S]);
    const int px = wave * 32 + r;
    const bool own = valid && yy >= y0 && yy < y0 + TH && gxm >= x0 && gxm < x0 + TW;
    const int o1 = own ? (int)((img + (long)yy * W + gxm) * (4 * C)) : OOB;
    if (px < LW) {
      float* slot = ring + (k & 3) * ROWF;
      const int key = qkey<PXT>(px);
      // the row inside the image and the tile's ring columns x0 - 1 .. x0 + TW too (uniform): no per-value select
      const bool interior = yy >= 0 && yy < H && x0 >= 1 && x0 + TW + 1 <= W;
      auto put = [&](auto masked_c) {
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f2v lo = round2<T>(f2v{acc[t][4 * g], acc[t][4 * g + 1]} + f2v{cw.bias[t][g][0], cw.bias[t][g][1]});
            const f2v hi = round2<T>(f2v{acc[t][4 * g + 2], acc[t][4 * g + 3]} + f2v{cw.bias[t][g][2], cw.bias[t][g][3]});
            float4 v = make_float4(lo.x, lo.y, hi.x, hi.y);
            if constexpr (decltype(masked_c)::value) v = valid ? v : f4(0.f);
            *reinterpret_cast<float4*>(slot + (px * 16 + ((8 * t + 2 * g + hh) ^ key)) * 4) = v;
          }
      };
      if (interior) put(std::false_type{});
      else put(std::true_type{});
    }
    if constexpr (KEEP) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          vec_t<T, 4> o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = (T)(acc[t][4 * g + q] + cw.bias[t][g][q]);
          bstore4<T>(r1, o1 + 2 * ((t == 0 ? 0 : C) + slice * 32 + 8 * g + 4 * hh), o);
        }
    }
  };

  float4 pacc = f4(0.f);
  // one output row: MFMA of ring row rr + 2 (slot S), barrier, depthwise of image row y0 + rr from ring rows rr .. rr + 2
  auto step = [&](auto slot_c, int rr) {
    __builtin_amdgcn_sched_barrier(0);  // no scheduling across steps
    if (mfma_wave) mfma_row(slot_c, rr + 2);
    lds_barrier();
    const int y = y0 + rr;
    f2v a2[PXT][2];
#pragma unroll
    for (int j = 0; j < PXT; ++j) {
      a2[j][0] = f2v{dw.b.x, dw.b.y};
      a2[j][1] = f2v{dw.b.z, dw.b.w};
    }
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float* row = ring + ((rr + dy) & 3) * ROWF;
      f2v xw[PXT + 2][2];
#pragma unroll
      for (int c = 0; c < PXT + 2; ++c) {
        const int px = xl + c;
        const float4 v = *reinterpret_cast<const float4*>(row + (px * 16 + (q16 ^ qkey<PXT>(px))) * 4);
        xw[c][0] = f2v{v.x, v.y};
        xw[c][1] = f2v{v.z, v.w};
      }
#pragma unroll
      for (int j = 0; j < PXT; ++j)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int e = 0; e < 2; ++e) a2[j][e] = __builtin_elementwise_fma(dw.w[dy * 3 + dx][e], xw[j + dx][e], a2[j][e]);
    }
#pragma unroll
    for (int j = 0; j < PXT; ++j) {
      const int gx = x0 + xl + j;
      const bool ok = y < H && gx < W;
      const float4 mine = f4of(a2[j]);
      const float4 other = swap32(mine, false);  // the partner quad's t2 (lane ^ 32; consumed by the gate lanes only)
      const long m = img + (long)y * W + gx;
      if constexpr (KEEP) bstore4<T>(r2, ok ? (int)(m * 4 * C) + 2 * ch : OOB, mine);
      float4 gv = mine * other;
      // the fp32 product is what is rounded to the storage type (the SimpleGate convention of every kernel)
      asm volatile("" : "+v"(gv.x), "+v"(gv.y), "+v"(gv.z), "+v"(gv.w));
      bstore4<T>(rg, ok && gate ? (int)(m * 2 * C) + 2 * ch : OOB, gv);
      if (ok) pacc += gv;
    }
  };

  if (mfma_wave) {
    mfma_row(IC<0>{}, 0);
    mfma_row(IC<1>{}, 1);
  }
#pragma unroll 1
  for (int rr = 0; rr < TH; rr += NR) {  // ring row rr + 2 lives in register slot (rr + 2) % NR
    step(IC<2>{}, rr);
    step(IC<3>{}, rr + 1);
    step(IC<0>{}, rr + 2);
    step(IC<1>{}, rr + 3);
  }
  // pool partial of the tile: the gate lanes of one quad (lane bits 3..4), then the 4 waves in order
#pragma unroll
  for (int o = 8; o < 32; o <<= 1) {
    pacc.x += __shfl_xor(pacc.x, o, 64); pacc.y += __shfl_xor(pacc.y, o, 64);
    pacc.z += __shfl_xor(pacc.z, o, 64); pacc.w += __shfl_xor(pacc.w, o, 64);
  }
  lds_barrier();  // the ring is dead
  if (lane < 8) st4(ring + (wave * 8 + lane) * 4, pacc);
  lds_barrier();
  if (tid < 32) {
    const int q = tid >> 2, e = tid & 3;
    const float s = ((ring[(0 * 8 + q) * 4 + e] + ring[(1 * 8 + q) * 4 + e]) + ring[(2 * 8 + q) * 4 + e]) +
                    ring[(3 * 8 + q) * 4 + e];
    p.pool[((long)b * p.tiles + tile) * C + slice * 32 + tid] = s;
  }
}

// ---------------------------------------------------------------- backward
// Geometry: a TH x TW (TW 32) tile of dt1 x one 32-gate-channel slice; t1 ring rows k = image row y0 - 2 + k (k 0 ..
// TH + 3, pixels x0 - 2 .. x0 + TW + 1), dt2 rows i = image row y0 - 1 + i (i 0 .. TH + 1, pixels x0 - 1 .. x0 + TW).
// Step j: barrier(j), then
//   B  dt1 of dt2-row o = j - 2 (1 <= o <= TH: image row y0 - 1 + o) from dt2 rows o - 1 .. o + 1, stored
//   C  dt2 row i = j: t2 = depthwise(t1 rows j .. j + 2) rounded; dg = dh a + ds / HW; dt2 = (dg t2[partner], ...)
//      rounded into the dt2 ring; for the tile's own rows dW2 += dt2 * window, db2 += dt2
//   A  (MFMA waves) t1 row j + 3
// Between two barriers the phases touch disjoint slots of the two 4-slot rings: B reads dt2 rows j - 3 .. j - 1
// (written by C before barrier(j)); C reads t1 rows j .. j + 2 (row j + 2 written by A before barrier(j)) and writes
// dt2 row j into the slot of row j - 4 (last read by B before barrier(j)); A writes t1 row j + 3 into the slot of row
// j - 1 (last read by C before barrier(j)).  B and C carry no branch: rows outside the tile are masked (dt2 zeroed,
// dt1 stores to an out-of-range offset).
// Both rings hold fp32 quads keyed as the forward's ring (rowring.h): the t1 ring the rounded t1 widened once, the dt2
// ring the rounded dt2 widened once (no conversions in the dt1 taps).  The conv1 weight slice and bias live in LDS; the
// n1 rows (MFMA waves) and the dh rows of the next steps in register rings with static slots (the step loop unrolled by
// the ring depth U: 3 at C 32, 2 at C 64).
// BAL: the t1 rebuild spread over all four waves (wave w: pixel chunk w / 2, channel half w % 2 -- one 32 x 32 MFMA
// chain and a 16-value epilogue each) instead of waves 0 / 1 doing both halves of one chunk each (two chains, 32
// values) while waves 2 / 3 wait at the step's barrier
template <typename T, int C, int TH, bool BAL, bool SCA = false>
__global__ __launch_bounds__(256, 2) void c1dw_bwd_tile(C1TileP p) {
  constexpr int TW = 32, PXT = 2, LT = TW + 4, LD = TW + 2, KS = C / 16, NSL = C / 32;
  constexpr int ROWF = LT * 64;          // floats per t1 ring row
  constexpr int ROWD = LD * 64;          // floats per dt2 ring row
  constexpr int U = 2;                   // register-ring slots (n1, dh); the step loop is unrolled by 4 = the LDS
                                         // rings' depth, so every ring and register slot is a compile-time index
  constexpr int RPB = 256 / (C * 2);     // weight rows per 256-byte LDS bank row (the swizzle key's divisor)
  constexpr int NC = 2 * KS;             // 16-byte chunks per weight row
  __shared__ __attribute__((aligned(16))) float t1r[4 * ROWF];
  __shared__ __attribute__((aligned(16))) float dt2r[4 * ROWD];
  __shared__ __attribute__((aligned(16))) T w1s[64 * C];
  __shared__ __attribute__((aligned(16))) float b1s[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int u = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = u % NSL, tile = (u / NSL) % p.tiles, b = u / (NSL * p.tiles);
  const int y0 = (tile / p.tiles_x) * TH, x0 = (tile % p.tiles_x) * TW;
  const int H = p.H, W = p.W;
  const long img = (long)b * H * W, M = (long)p.B * H * W;
  const __amdgpu_buffer_rsrc_t rn = rsrc(p.n1, M * C * 2), rh = rsrc(p.dh, M * C * 2), ro = rsrc(p.dt1, M * C * 4);
  // ---- SCA: ds of the slice's 32 gate channels from the channel-dot partials (sca_bwd.h), first, while nothing else
  // is live; scratch in the dt2 ring (first written after step 0's barrier): part | da | GEMV partials | ds
  [[maybe_unused]] const ScaBwdP sq{p.da_slab, p.wsca, p.mean, p.dwsca, p.dbsca, p.chunks, p.B, C};
  static_assert(!SCA || 3072 + 32 <= 4 * ROWD, "SCA scratch");
  if constexpr (SCA) sca_ds_slice<256, 32>(sq, b, slice * 32, dt2r, dt2r + 1024, dt2r + 2048, dt2r + 3072);
  // ---- the slice's conv1 weight rows (n = t * 32 + rr) and bias into LDS; chunk c of row n at c ^ key(n)
  {
    const T* w1 = reinterpret_cast<const T*>(p.w1);
    for (int i = tid; i < 64 * NC; i += 256) {
      const int n = i / NC, c = i % NC;
      const int grow = (n < 32 ? 0 : C) + slice * 32 + (n & 31);
      const uint4 v = *reinterpret_cast<const uint4*>(w1 + (long)grow * C + 8 * c);
      *reinterpret_cast<uint4*>(w1s + n * C + 8 * (c ^ ((n / RPB) & (NC - 1)))) = v;
    }
    if (tid < 64) b1s[tid] = p.b1[(tid < 32 ? 0 : C) + slice * 32 + (tid & 31)];
  }
  // ---- MFMA lanes: waves 0 and 1, chunk = wave (t1 ring pixel wave * 32 + r = image column x0 - 2 + ...); BAL: every
  // wave, chunk = wave / 2, channel half th = wave % 2
  const bool mfma_wave = BAL || wave < 2;
  const int chunk = BAL ? wave >> 1 : wave, th = wave & 1;
  const int gxm = x0 - 2 + chunk * 32 + r;
  const bool lane_ok = chunk * 32 + r < LT;
  vec_t<T, 8> fq[U][KS];  // n1 fragments of t1 ring row k in slot k % U
  if (mfma_wave)
#pragma unroll
    for (int k = 0; k < U; ++k) load_n1<T, KS>(rn, img, W, H, y0 - 2 + k, gxm, lane_ok, hh, fq[k]);
  // ---- depthwise lanes: quad q16 at tile columns xl, xl + 1 (dt2 ring pixels xl + 1, xl + 2); the 32 lanes of
  // column group 0 of waves 2 / 3 (no MFMA phase) also own the halo pixel of the dt2 rows (ring pixel 0 / TW + 1)
  const int q16 = (lane & 7) + 8 * hh, xl = PXT * (4 * wave + ((lane >> 3) & 3));
  const bool gate = hh == 0;
  const int ch = (gate ? 0 : C) + slice * 32 + 4 * (lane & 7);  // conv channels of this lane
  const int gch = slice * 32 + 4 * (lane & 7);                 // their gate channels (dg, dh)
  const bool has_halo = wave >= 2 && ((lane >> 3) & 3) == 0;
  const int dph = wave == 2 ? 0 : TW + 1;
  DwQuad dw;
  dw.load(p.wdw, p.bdw, ch);
  const float4 ak = ld4(p.a + (long)b * C + gch);
  const float4 sk = (SCA ? ld4(dt2r + 3072 + 4 * (lane & 7)) : ld4(p.ds + (long)b * C + gch)) * f4(p.inv_hw);
  auto dh_off = [&](int yy, int gx, bool lane_has) {
    return lane_has && yy >= 0 && yy < H && gx >= 0 && gx < W ? (int)((img + (long)yy * W + gx) * (2 * C)) + 2 * gch : OOB;
  };
  vec_t<T, 4> dq[U][PXT], dqh[U];  // dh of dt2 row i in slot i % U
#pragma unroll
  for (int k = 0; k < U; ++k) {
#pragma unroll
    for (int j = 0; j < PXT; ++j) dq[k][j] = bload4<T>(rh, dh_off(y0 - 1 + k, x0 + xl + j, true));
    dqh[k] = bload4<T>(rh, dh_off(y0 - 1 + k, x0 - 1 + dph, has_halo));
  }
  f2v aw[9][2], db[2];  // this lane's depthwise weight / bias gradient partials
#pragma unroll
  for (int t = 0; t < 9; ++t) aw[t][0] = aw[t][1] = f2v{0.f, 0.f};
  db[0] = db[1] = f2v{0.f, 0.f};
  lds_barrier();  // weight slice and bias in LDS

  // A: t1 ring row k (image row y0 - 2 + k) from register slot S = k % U, which then takes row k + U
  auto mfma_row = [&](auto slot_c, auto ring_c, int k) {
    constexpr int S = decltype(slot_c)::value;  // k % U
    constexpr int R = decltype(ring_c)::value;  // k & 3
    const int yy = y0 - 2 + k;
    if (k <= TH + 3) {  // uniform
      const bool valid = yy >= 0 && yy < H && lane_ok && gxm >= 0 && gxm < W;
      // the row inside the image and the tile's ring columns x0 - 2 .. x0 + TW + 1 too (uniform): no per-value select
      const bool interior = yy >= 0 && yy < H && x0 >= 2 && x0 + TW + 2 <= W;
      constexpr int NT = BAL ? 1 : 2;  // channel halves of this wave
      floatx16 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int n = (BAL ? th : t) * 32 + r, c = 2 * ks + hh;
          const vec_t<T, 8> wf = *reinterpret_cast<const vec_t<T, 8>*>(w1s + n * C + 8 * (c ^ ((n / RPB) & (NC - 1))));
          acc[t] = mfma32x32x16(wf, fq[S][ks], acc[t]);
        }
      const int px = chunk * 32 + r;
      if (px < LT) {
        float* slot = t1r + R * ROWF;
        const int key = qkey<PXT>(px);
        auto put = [&](auto masked_c) {
#pragma unroll
          for (int t0 = 0; t0 < NT; ++t0)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int t = BAL ? th : t0;
              const float4 bv = *reinterpret_cast<const float4*>(b1s + t * 32 + 8 * g + 4 * hh);
              const f2v lo = round2<T>(f2v{acc[t0][4 * g], acc[t0][4 * g + 1]} + f2v{bv.x, bv.y});
              const f2v hi = round2<T>(f2v{acc[t0][4 * g + 2], acc[t0][4 * g + 3]} + f2v{bv.z, bv.w});
              float v[4] = {lo.x, lo.y, hi.x, hi.y};
              if constexpr (decltype(masked_c)::value) {
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] = valid ? v[q] : 0.f;
              }
              *reinterpret_cast<float4*>(slot + (px * 16 + ((8 * t + 2 * g + hh) ^ key)) * 4) =
                  make_float4(v[0], v[1], v[2], v[3]);
            }
        };
        if (interior) put(std::false_type{});
        else put(std::true_type{});
      }
    }
    load_n1<T, KS>(rn, img, W, H, yy + U, gxm, lane_ok, hh, fq[S]);  // OOB past the image: zeros, no branch
  };

  // C: dt2 of this lane's quad at NP adjacent dt2 ring pixels dp0 .. (image columns x0 - 1 + dp) of dt2 row i, from t1
  // ring rows i .. i + 2; own_row: accumulate the depthwise weight / bias gradients of the tile's own pixels
  auto dt2_px = [&](auto np_c, auto own_c, auto ring_c, int dp0, int i, const vec_t<T, 4>* dv, float* drow, float own) {
    constexpr int RI = decltype(ring_c)::value;  // i & 3
    constexpr int NP = decltype(np_c)::value;
    constexpr bool OWN = decltype(own_c)::value;
    const int yd = y0 - 1 + i;
    const bool row_in = yd >= 0 && yd < H && i <= TH + 1;
    f2v a2[NP][2];
    f2v xw[3][NP + 2][2];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      a2[j][0] = f2v{dw.b.x, dw.b.y};
      a2[j][1] = f2v{dw.b.z, dw.b.w};
    }
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float* row = t1r + ((RI + dy) & 3) * ROWF;
#pragma unroll
      for (int c = 0; c < NP + 2; ++c) {
        const int px = dp0 + c;  // t1 ring pixel (image column x0 - 2 + px)
        const float4 v = *reinterpret_cast<const float4*>(row + (px * 16 + (q16 ^ qkey<PXT>(px))) * 4);
        xw[dy][c][0] = f2v{v.x, v.y};
        xw[dy][c][1] = f2v{v.z, v.w};
      }
#pragma unroll
      for (int j = 0; j < NP; ++j)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int e = 0; e < 2; ++e) a2[j][e] = __builtin_elementwise_fma(dw.w[dy * 3 + dx][e], xw[dy][j + dx][e], a2[j][e]);
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int dp = dp0 + j, gx = x0 - 1 + dp;
      const bool inside = row_in && gx >= 0 && gx < W;
      const f2v m0 = round2<T>(a2[j][0]), m1 = round2<T>(a2[j][1]);
      const float4 mine = make_float4(m0.x, m0.y, m1.x, m1.y);  // t2 rounded
      const float4 other = swap32(mine, hh);  // the partner quad's rounded t2 (lane ^ 32)
      const float oth[4] = {other.x, other.y, other.z, other.w};
      const float av[4] = {ak.x, ak.y, ak.z, ak.w}, sv[4] = {sk.x, sk.y, sk.z, sk.w};
      float pr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dg = fmaf((float)dv[j][e], av[e], sv[e]);
        pr[e] = dg * oth[e];
        asm volatile("" : "+v"(pr[e]));  // the fp32 product is what is rounded (the fused depthwise backward's convention)
      }
      const f2v r0 = round2<T>(f2v{pr[0], pr[1]}), r1 = round2<T>(f2v{pr[2], pr[3]});
      const float d2[4] = {inside ? r0.x : 0.f, inside ? r0.y : 0.f, inside ? r1.x : 0.f, inside ? r1.y : 0.f};
      *reinterpret_cast<float4*>(drow + (dp * 16 + (q16 ^ qkey<PXT>(dp))) * 4) = make_float4(d2[0], d2[1], d2[2], d2[3]);
      if constexpr (OWN) {  // own (uniform 0 / 1): the dt2 row is one of the tile's; d2 is 0 outside the image
        const f2v l0 = f2v{d2[0], d2[1]} * own, l1 = f2v{d2[2], d2[3]} * own;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          aw[t][0] = __builtin_elementwise_fma(l0, xw[t / 3][j + t % 3][0], aw[t][0]);
          aw[t][1] = __builtin_elementwise_fma(l1, xw[t / 3][j + t % 3][1], aw[t][1]);
        }
        db[0] += l0;
        db[1] += l1;
      }
    }
  };

  // the halo dt2 pixel of waves 2 / 3 (ring pixel dph of dt2 row i): t2, the partner's t2, dt2 into the ring; no
  // weight-gradient terms (it is not one of the tile's pixels)
  auto halo_dt2 = [&](auto ring_c, int i, const vec_t<T, 4>& dv, float* drow) {
    constexpr int RI = decltype(ring_c)::value;  // i & 3
    const int yd = y0 - 1 + i, gx = x0 - 1 + dph;
    const bool inside = yd >= 0 && yd < H && i <= TH + 1 && gx >= 0 && gx < W;
    f2v a0 = f2v{dw.b.x, dw.b.y}, a1 = f2v{dw.b.z, dw.b.w};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const float* row = t1r + ((RI + dy) & 3) * ROWF;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int px = dph + dx;
        const float4 v = *reinterpret_cast<const float4*>(row + (px * 16 + (q16 ^ qkey<PXT>(px))) * 4);
        a0 = __builtin_elementwise_fma(dw.w[dy * 3 + dx][0], f2v{v.x, v.y}, a0);
        a1 = __builtin_elementwise_fma(dw.w[dy * 3 + dx][1], f2v{v.z, v.w}, a1);
      }
    }
    const f2v m0 = round2<T>(a0), m1 = round2<T>(a1);
    const float4 other = swap32(make_float4(m0.x, m0.y, m1.x, m1.y), hh);
    const float oth[4] = {other.x, other.y, other.z, other.w};
    const float av[4] = {ak.x, ak.y, ak.z, ak.w}, sv[4] = {sk.x, sk.y, sk.z, sk.w};
    float pr[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      pr[e] = fmaf((float)dv[e], av[e], sv[e]) * oth[e];
      asm volatile("" : "+v"(pr[e]));
    }
    const f2v r0 = round2<T>(f2v{pr[0], pr[1]}), r1 = round2<T>(f2v{pr[2], pr[3]});
    *reinterpret_cast<float4*>(drow + (dph * 16 + (q16 ^ qkey<PXT>(dph))) * 4) =
        inside ? make_float4(r0.x, r0.y, r1.x, r1.y) : f4(0.f);
    // the weight-gradient partials pass through this branch untouched; naming them here (no instruction) keeps the
    // register allocation of the unconditional path (without it the compiler spills 250+ VGPRs)
#pragma unroll
    for (int t = 0; t < 10; ++t)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f2v v = t < 9 ? aw[t][e] : db[e];
        asm volatile("" : "+v"(v));
        if (t < 9) aw[t][e] = v;
        else db[e] = v;
      }
  };

  // step j (see the geometry above): barrier(j); B: dt1 of dt2-row j - 2; C: dt2 row j; A: t1 row j + 3
  auto step = [&](auto j_c, int j) {
    constexpr int J = decltype(j_c)::value;  // j = 4 m + J: ring slot of dt2 row j; dh register slot J % U
    __builtin_amdgcn_sched_barrier(0);       // no scheduling across steps (it hoists later steps' loads: spills)
    lds_barrier();
    // B: dt1 of dt2-row o = j - 2 (image row y0 - 1 + o) from dt2 rows o - 1 .. o + 1
    {
      const int o = j - 2, yo = y0 - 1 + o;
      const bool orow = o >= 1 && o <= TH && yo < H;
      f2v acc[PXT][2];
#pragma unroll
      for (int jj = 0; jj < PXT; ++jj) acc[jj][0] = acc[jj][1] = f2v{0.f, 0.f};
#pragma unroll
      for (int dhh = -1; dhh <= 1; ++dhh) {
        const float* dr = dt2r + ((J + 2 - dhh) & 3) * ROWD;  // tap (dhh, dww): dt2 row o - dhh, ring pixel p + 1 - dww
        f2v gw[PXT + 2][2];
#pragma unroll
        for (int c = 0; c < PXT + 2; ++c) {
          const int dp = xl + c;
          const float4 v = *reinterpret_cast<const float4*>(dr + (dp * 16 + (q16 ^ qkey<PXT>(dp))) * 4);
          gw[c][0] = f2v{v.x, v.y};
          gw[c][1] = f2v{v.z, v.w};
        }
#pragma unroll
        for (int jj = 0; jj < PXT; ++jj)
#pragma unroll
          for (int dww = -1; dww <= 1; ++dww) {
            const int t = (dhh + 1) * 3 + (dww + 1);
#pragma unroll
            for (int e = 0; e < 2; ++e) acc[jj][e] = __builtin_elementwise_fma(dw.w[t][e], gw[jj + 1 - dww][e], acc[jj][e]);
          }
      }
#pragma unroll
      for (int jj = 0; jj < PXT; ++jj) {
        const int gx = x0 + xl + jj;
        bstore4<T>(ro, orow && gx < W ? (int)((img + (long)yo * W + gx) * (4 * C)) + 2 * ch : OOB, f4of(acc[jj]));
      }
    }
    // C: dt2 row i = j
    {
      const int i = j, yd = y0 - 1 + i;
      float* drow = dt2r + J * ROWD;
      dt2_px(IC<PXT>{}, std::true_type{}, IC<J>{}, xl + 1, i, dq[J % U], drow, i >= 1 && i <= TH ? 1.f : 0.f);
      if (has_halo) halo_dt2(IC<J>{}, i, dqh[J % U], drow);
#pragma unroll
      for (int jj = 0; jj < PXT; ++jj) dq[J % U][jj] = bload4<T>(rh, dh_off(yd + U, x0 + xl + jj, true));
      dqh[J % U] = bload4<T>(rh, dh_off(yd + U, x0 - 1 + dph, has_halo));
    }
    // A: t1 ring row j + 3 (register slot (j + 3) % U)
    if (mfma_wave) mfma_row(IC<(J + 3) % U>{}, IC<(J + 3) & 3>{}, j + 3);
  };

  if (mfma_wave) {  // t1 ring rows 0 .. 2 (register slots k % U)
    mfma_row(IC<0>{}, IC<0>{}, 0);
    mfma_row(IC<1 % U>{}, IC<1>{}, 1);
    mfma_row(IC<2 % U>{}, IC<2>{}, 2);
  }
  static_assert(U == 2, "register ring depth (divides the unroll of 4)");
  constexpr int NS = TH + 3;  // steps j = 0 .. TH + 2: C(j) to dt2 row TH + 1, B(j + 1) to dt1 row TH
#pragma unroll 1
  for (int j = 0; j < NS - NS % 4; j += 4) {
    step(IC<0>{}, j);
    step(IC<1>{}, j + 1);
    step(IC<2>{}, j + 2);
    step(IC<3>{}, j + 3);
  }
  if constexpr (NS % 4 >= 1) step(IC<0>{}, NS - NS % 4);
  if constexpr (NS % 4 >= 2) step(IC<1>{}, NS - NS % 4 + 1);
  if constexpr (NS % 4 >= 3) step(IC<2>{}, NS - NS % 4 + 2);
  // ---- the tile's depthwise weight / bias gradients: 40 values per lane, summed over the lanes of one quad (lane bits
  // 3..4: a reduce-scatter, 40 -> 20 -> 10 values per lane), then over the 4 waves in order
  float v[40];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    v[4 * t + 0] = aw[t][0].x; v[4 * t + 1] = aw[t][0].y; v[4 * t + 2] = aw[t][1].x; v[4 * t + 3] = aw[t][1].y;
  }
  v[36] = db[0].x; v[37] = db[0].y; v[38] = db[1].x; v[39] = db[1].y;
  float v2[20], v3[10];
  const bool b3 = lane & 8, b4 = lane & 16;
#pragma unroll
  for (int j = 0; j < 20; ++j) {
    const float snd = b3 ? v[j] : v[j + 20], keep = b3 ? v[j + 20] : v[j];
    v2[j] = keep + __shfl_xor(snd, 8, 64);
  }
#pragma unroll
  for (int j = 0; j < 10; ++j) {
    const float snd = b4 ? v2[j] : v2[j + 10], keep = b4 ? v2[j + 10] : v2[j];
    v3[j] = keep + __shfl_xor(snd, 16, 64);
  }
  lds_barrier();  // the t1 ring is dead: the cross-wave buffer [wave][q16][40]
  float* red = t1r;
  const int e0 = (b3 ? 20 : 0) + (b4 ? 10 : 0);
#pragma unroll
  for (int j = 0; j < 10; ++j) red[(wave * 16 + q16) * 40 + e0 + j] = v3[j];
  lds_barrier();
  const long row = (long)b * p.tiles + tile;
  for (int i = tid; i < 16 * 40; i += 256) {
    const int qq = i / 40, e = i % 40;
    const float s = ((red[(0 * 16 + qq) * 40 + e] + red[(1 * 16 + qq) * 40 + e]) + red[(2 * 16 + qq) * 40 + e]) +
                    red[(3 * 16 + qq) * 40 + e];
    const int c4 = ((qq < 8) ? 0 : C) + slice * 32 + 4 * (qq & 7);
    if (e < 36) p.slab_w[(row * 2 * C + c4 + (e & 3)) * 9 + (e >> 2)] = s;
    else p.slab_b[row * 2 * C + c4 + (e - 36)] = s;
  }
  if constexpr (SCA) sca_dw_rows<256>(sq, dt2r, dt2r + SCA_DW_BMAX);  // (the dt2 ring is dead; its first barrier)
}

}  // namespace
}  // namespace nbp

using namespace nbp;

namespace {
int tile_w(int C) { return C == 32 ? 64 : 32; }
// rows of a backward tile: 32 (the two-row halo of the rebuilt t1 and the one-row halo of the rebuilt t2 are then
// 1.125 / 1.06 x the tile's rows instead of 1.25 / 1.125 at 16, and the per-tile weight-slice load and dW reduction
// amortise over twice the pixels); NBP_C1DW_BWD_TH=16 / 32 (per C: "th32,th64") overrides for A/B runs; 64 at level 0
// (512 workgroups: one resident round) measured 148.3 -> 141.1 us per launch in scripts/c1dw_tile_micro.py but
// neutral-to-negative in the step (1476.8 / 1470.7 vs 1479.3 / 1474.1 img/s, gpurun_out r6v): not the default
// the balanced t1 rebuild (BAL) at C 32: 151.0 -> 148.7-149.4 us per level-0 launch (scripts/c1dw_tile_micro.py,
// gpurun_out r6c); at C 64 its registers spill (256 VGPRs + 10) and it is slower (89.1 -> 93.3 us): off there.
// NBP_C1DW_BWD_BAL=0 / 1 forces it off / on at both (A/B)
bool bwd_bal(int C) {
  static const int v = [] {
    const char* e = getenv("NBP_C1DW_BWD_BAL");
    return e ? atoi(e) : -1;
  }();
  return v < 0 ? C == 32 : v != 0;
}
int bwd_th(int C) {
  static int th[2] = {0, 0};
  if (!th[0]) {
    th[0] = th[1] = 32;
    if (const char* e = getenv("NBP_C1DW_BWD_TH")) {
      int a = 0, b = 0;
      const int n = sscanf(e, "%d,%d", &a, &b);
      if (n >= 1 && (a == 16 || a == 32 || a == 64)) th[0] = a;  // 64: level 0 (C 32) only
      if (n >= 1 && (a == 16 || a == 32)) th[1] = a;
      if (n == 2 && (b == 16 || b == 32)) th[1] = b;
    }
  }
  return th[C == 32 ? 0 : 1];
}
}  // namespace

extern "C" {

int nbp_c1dw_tile_supported(int B, int H, int W, int C, int dtype) {
  if (dtype != 1 && dtype != 2) return 0;
  if (C != 32 && C != 64) return 0;
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  // every buffer the kernels address (the largest: t1 / t2 / dt1, [M][2C] 16-bit = M * C * 4 bytes) by 32-bit buffer
  // offsets, with OOB past its end: a masked access must fall outside the range (larger levels take the stored tape)
  return (long)B * H * W * C * 4 <= (long)OOB ? 1 : 0;
}

int nbp_c1dw_tile_rows(int H, int W, int C) {
  if (C != 32 && C != 64) return 0;
  return cdiv(H, CT_TH) * cdiv(W, tile_w(C));
}

int nbp_c1dw_fwd_tile(const void* n1, const void* w1, const float* b1, const float* wdw, const float* bdw, void* t1,
                      void* t2, void* g, float* pool_slab, int B, int H, int W, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(n1 && w1 && b1 && wdw && bdw && g && pool_slab && B > 0, "nbp_c1dw_fwd_tile: null pointer");
  NBP_REQUIRE(nbp_c1dw_tile_supported(B, H, W, C, dtype),
              "nbp_c1dw_fwd_tile: unsupported shape (B %d H %d W %d C %d dtype %d; B*H*W*2C*2 bytes must not exceed "
              "the out-of-range buffer offset)", B, H, W, C, dtype);
  const int tw = tile_w(C);
  C1TileP p{};
  p.n1 = n1; p.w1 = w1; p.b1 = b1; p.wdw = wdw; p.bdw = bdw; p.t1 = t1; p.t2 = t2; p.g = g; p.pool = pool_slab;
  p.B = B; p.H = H; p.W = W; p.tiles_x = cdiv(W, tw); p.tiles = nbp_c1dw_tile_rows(H, W, C);
  const long nblk = (long)B * p.tiles * (C / 32);
  NBP_REQUIRE(nblk < (1L << 31), "nbp_c1dw_fwd_tile: grid too large");
  NBP_REQUIRE((t1 == nullptr) == (t2 == nullptr), "nbp_c1dw_fwd_tile: t1 and t2 are kept together or not at all");
  const bool keep = t1 != nullptr;
  NBP_DISPATCH_H(dtype, {
    if (C == 32) {
      if (keep) c1dw_fwd_tile<H, 32, 64, true><<<nblk, 256, 0, S(s)>>>(p);
      else c1dw_fwd_tile<H, 32, 64, false><<<nblk, 256, 0, S(s)>>>(p);
    } else {
      if (keep) c1dw_fwd_tile<H, 64, 32, true><<<nblk, 256, 0, S(s)>>>(p);
      else c1dw_fwd_tile<H, 64, 32, false><<<nblk, 256, 0, S(s)>>>(p);
    }
  });
  return check_launch("c1dw_fwd_tile");
}

size_t nbp_c1dw_bwd_workspace_floats(int B, int H, int W, int C) {
  return (size_t)B * cdiv(H, bwd_th(C)) * cdiv(W, 32) * 2 * C * 10;
}

}  // extern "C"

namespace {
int c1dw_bwd_launch(const void* dh, const float* a, const float* ds, const void* n1, const void* w1, const float* b1,
                    const float* wdw, const float* bdw, void* dt1, float* dwdw, float* dbdw, float* ws, int B, int H,
                    int W, int C, int dtype, nbp_stream_t s, const ScaBwdP* sca) {
  NBP_REQUIRE(dh && a && (ds || sca) && n1 && w1 && b1 && wdw && bdw && dt1 && dwdw && dbdw && ws && B > 0,
              "nbp_c1dw_bwd_tile: null pointer");
  NBP_REQUIRE(nbp_c1dw_tile_supported(B, H, W, C, dtype),
              "nbp_c1dw_bwd_tile: unsupported shape (B %d H %d W %d C %d dtype %d; B*H*W*2C*2 bytes must not exceed "
              "the out-of-range buffer offset)", B, H, W, C, dtype);
  C1TileP p{};
  p.n1 = n1; p.w1 = w1; p.b1 = b1; p.wdw = wdw; p.bdw = bdw; p.dh = dh; p.a = a; p.ds = ds; p.dt1 = dt1;
  const int th = bwd_th(C);
  p.B = B; p.H = H; p.W = W; p.tiles_x = cdiv(W, 32); p.tiles = cdiv(H, th) * p.tiles_x;
  p.inv_hw = 1.f / (float)((long)H * W);
  if (sca) {
    p.da_slab = sca->da_slab; p.wsca = sca->wsca; p.mean = sca->mean; p.dwsca = sca->dwsca; p.dbsca = sca->dbsca;
    p.chunks = sca->chunks;
  }
  const long nrow = (long)B * p.tiles;
  p.slab_w = ws;
  p.slab_b = ws + nrow * 2 * C * 9;
  const long nblk = nrow * (C / 32);
  NBP_REQUIRE(nblk < (1L << 31), "nbp_c1dw_bwd_tile: grid too large");
  const bool bal = bwd_bal(C);
  // the SCA fold is instantiated for the default variants (TH 32; the balanced rebuild at C 32 only)
  NBP_REQUIRE(!sca || (th == 32 && bal == (C == 32)),
              "nbp_sca_c1dw_bwd_tile: the SCA fold needs the default tile variant (NBP_C1DW_BWD_TH / _BAL unset)");
  lt_begin(S(s));
  NBP_DISPATCH_H(dtype, {
    if (sca && C == 32) c1dw_bwd_tile<H, 32, 32, true, true><<<nblk, 256, 0, S(s)>>>(p);
    else if (sca) c1dw_bwd_tile<H, 64, 32, false, true><<<nblk, 256, 0, S(s)>>>(p);
    else if (C == 32 && th == 64 && bal) c1dw_bwd_tile<H, 32, 64, true><<<nblk, 256, 0, S(s)>>>(p);
    else if (C == 32 && th == 64) c1dw_bwd_tile<H, 32, 64, false><<<nblk, 256, 0, S(s)>>>(p);
    else if (C == 32 && th == 32 && bal) c1dw_bwd_tile<H, 32, 32, true><<<nblk, 256, 0, S(s)>>>(p);
    else if (C == 32 && th == 32) c1dw_bwd_tile<H, 32, 32, false><<<nblk, 256, 0, S(s)>>>(p);
    else if (C == 32) c1dw_bwd_tile<H, 32, 16, false><<<nblk, 256, 0, S(s)>>>(p);
    else if (th == 32 && bal) c1dw_bwd_tile<H, 64, 32, true><<<nblk, 256, 0, S(s)>>>(p);
    else if (th == 32) c1dw_bwd_tile<H, 64, 32, false><<<nblk, 256, 0, S(s)>>>(p);
    else c1dw_bwd_tile<H, 64, 16, false><<<nblk, 256, 0, S(s)>>>(p);
  });
  {  // per-launch record (nbp_launch_timing): dh C + n1 C in, dt1 2C out, the conv1 weight slice per slice (+ SCA:
     // the channel-dot slab and W_sca read, dW_sca written)
    const double M = (double)B * H * W;
    const char* nm = sca ? (C == 32 ? "c1dw_bwd_tile<T,32,sca>" : "c1dw_bwd_tile<T,64,sca>")
                         : (C == 32 ? "c1dw_bwd_tile<T,32>" : "c1dw_bwd_tile<T,64>");
    const double sb = sca ? 4.0 * ((double)B * sca->chunks * C + 2.0 * C * C) : 0.0;
    lt_end(S(s), nm, 2.0 * M * 2 * C * C + 3 * 2.0 * M * 2 * C * 9 + (sca ? 4.0 * B * C * C : 0.0),
           (4.0 * M * C + 2.0 * C * C) * 2 + sb);
  }
  int rc = check_launch("c1dw_bwd_tile");
  if (rc) return rc;
  rc = nbp_reduce_slab(p.slab_w, (int)nrow, 2L * C * 9, dwdw, s);
  if (rc) return rc;
  return nbp_reduce_slab(p.slab_b, (int)nrow, 2L * C, dbdw, s);
}
}  // namespace

extern "C" {

int nbp_c1dw_bwd_tile(const void* dh, const float* a, const float* ds, const void* n1, const void* w1, const float* b1,
                      const float* wdw, const float* bdw, void* dt1, float* dwdw, float* dbdw, float* ws, int B, int H,
                      int W, int C, int dtype, nbp_stream_t s) {
  return c1dw_bwd_launch(dh, a, ds, n1, w1, b1, wdw, bdw, dt1, dwdw, dbdw, ws, B, H, W, C, dtype, s, nullptr);
}

int nbp_sca_c1dw_bwd_tile(const void* dh, const float* a, const float* da_slab, int chunks, const float* wsca,
                          const float* mean, float* dwsca, float* dbsca, const void* n1, const void* w1, const float* b1,
                          const float* wdw, const float* bdw, void* dt1, float* dwdw, float* dbdw, float* ws, int B,
                          int H, int W, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(da_slab && wsca && mean && dwsca && dbsca && chunks > 0, "nbp_sca_c1dw_bwd_tile: null pointer");
  NBP_REQUIRE(B <= SCA_DW_BMAX, "nbp_sca_c1dw_bwd_tile: B <= %d", SCA_DW_BMAX);
  const ScaBwdP q{da_slab, wsca, mean, dwsca, dbsca, chunks, B, C};
  return c1dw_bwd_launch(dh, a, nullptr, n1, w1, b1, wdw, bdw, dt1, dwdw, dbdw, ws, B, H, W, C, dtype, s, &q);
}

}  // extern "C"
