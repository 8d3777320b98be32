// Whole-image conv1 -> depthwise 3x3 -> SimpleGate -> pool partials at the deep U-Net levels (NAFNet_arch.py:59-68:
// conv1, conv2 (dw3x3), SimpleGate, the SCA's AdaptiveAvgPool2d) in ONE launch.
//
// At the 16 x 16 level (C 512) a whole image is one spatial tile, so the stencil needs no halo
// recompute: a workgroup owns (image b, a slice of GS gate channels c = cbase .. cbase + GS - 1 and their SimpleGate
// partners C + c).  Phase 1 is the conv1 GEMM of that slice, t1[HW x 2 GS] = n1[HW x C] . W1[slice rows]^T + b1, on
// 32x32x16 MFMA (8 waves, each 32 TM pixel rows x 2 GS columns; the weight slice in LDS, the pixel rows streamed from
// memory in fragment order with a register ring).  Phase 2 rounds t1 to the storage type into a zero-bordered LDS
// frame (the depthwise conv's zero padding) and stores it (the backward's tape).  Phase 3 runs the depthwise conv with
// rolling 3x3 register windows on packed pairs, the SimpleGate and the pool sum of the slice over the whole image.
//
// Bitwise contract: t1, t2 and g equal the two-launch path (gemm_glds_kernel conv1 + dw_sg_pool_tiled): the same MFMA
// sequence per t1 element (K ascending in steps of 16, one accumulator chain, + bias, one rounding), the same tap order
// per depthwise output (bias, then taps 0..8 by fused multiply-add) and the same opaque fp32 gate product.  The pool
// sum (the fp32 gate products of the image) is one fixed-order sum per channel instead of per-tile partials: equal to
// the two-launch value up to fp32 summation order.
#include "nbp_common.h"

namespace nbp {
namespace {

struct C1DwP {
  const void* n1;     // [B][HW][C] 16-bit: the block's norm1 output (conv1 input)
  const void* w1;     // [2C][C] 16-bit: conv1 weight (forward copy)
  const float* b1;    // [2C]
  const float* wdw;   // [2C][9]
  const float* bdw;   // [2C]
  void* t1;           // [B][HW][2C] out (tape)
  void* t2;           // [B][HW][2C] out (tape; may be null: no backward)
  void* g;            // [B][HW][C] out
  float* pool;        // [B][C] out: the pool sum of the gate products (a one-chunk pool slab)
  int B;
};

// C: block width; S: image side (H = W = S); NCH = 2 GS conv channels per workgroup
template <typename H, int C, int S, int NCH>
__global__ __launch_bounds__(512) void c1_dw_sg_pool_img(C1DwP p) {
  constexpr int HW = S * S, GS = NCH / 2, NW = 8;
  constexpr int TM = HW / (32 * NW), TN = NCH / 32;  // 32x32 MFMA tiles per wave (pixel rows x channels)
  static_assert(TM >= 1 && TN >= 1 && TM * 32 * NW == HW && TN * 32 == NCH, "tile shape");
  // the wave's pixel rows stream through a wave-private LDS-DMA ring (full 128-byte lines per DMA piece; no
  // workgroup barrier): KC K elements per stage, NSTG stages
  constexpr int KC = TM == 1 ? 64 : 16, RB = KC * 2, ROWS = 32 * TM, STG = ROWS * RB, NSTG = TM == 1 ? 3 : 4;
  constexpr int NST = C / KC;
  constexpr int PIECES = STG / 1024, RPP = 1024 / RB, SPR = RB / 16;  // DMA pieces per stage, rows / slots per piece
  static_assert(PIECES * 1024 == STG && NST >= NSTG, "ring geometry");
  constexpr int WROW = C * 2;                         // weight-slice row bytes in LDS
  constexpr int FW = S + 2;                           // frame row (pixels)
  constexpr int WS_BYTES = NCH * WROW, RING_BYTES = 8 * NSTG * STG, FR_BYTES = FW * FW * NCH * 2;
  constexpr int P1 = WS_BYTES + RING_BYTES, SM = P1 > FR_BYTES ? P1 : FR_BYTES;
  static_assert(SM <= 160 * 1024 && 512 * 16 <= FR_BYTES, "LDS");
  static_assert((C / 8) >= 16, "weight-slice swizzle: >= 16 chunks per row");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 31, h = lane >> 5;
  constexpr int SLICES = C / GS;
  // the slices of one image on one XCD (they all stream the image's n1 rows: L2 hits)
  const int u = xcd_remap(blockIdx.x, gridDim.x);
  const int slice = u % SLICES, b = u / SLICES;
  const int cbase = slice * GS;
  auto gch = [&](int n) { return n < GS ? cbase + n : C + cbase + (n - GS); };  // tile column -> conv channel
  const H* n1 = reinterpret_cast<const H*>(p.n1) + ((long)b * HW + wave * ROWS) * C;
  const H* w1 = reinterpret_cast<const H*>(p.w1);
  unsigned char* ring = smem + WS_BYTES + wave * NSTG * STG;
  // slot permutation of a ring row (the 16 rows a ds_read_b128 lane group reads hit distinct bank groups)
  auto swz = [](int row) { return SPR == 8 ? (row >> 1) & 7 : SPR == 4 ? (row >> 2) & 3 : (row >> 3) & 1; };
  // DMA piece q of stage t: lane l fills row q RPP + l / SPR, slot l % SPR with chunk slot ^ swz(row)
  const int prow = lane / SPR, pslot = lane % SPR;
  auto issue = [&](int t) {
#pragma unroll
    for (int q = 0; q < PIECES; ++q) {
      const int row = q * RPP + prow, c = pslot ^ swz(row);
      glds16(n1 + (long)row * C + t * KC + 8 * c, ring + (t % NSTG) * STG + q * 1024);
    }
  };
#pragma unroll
  for (int t = 0; t < NSTG - 1; ++t) issue(t);
  // ---- the weight slice into LDS: row n (tile column), 16-byte chunk k at slot k ^ (n & 15) (the 16 rows a
  // ds_read_b128 lane group reads at one chunk hit 16 distinct slots)
  {
    constexpr int CH = WROW / 16, TOT = NCH * CH, NI = (TOT + 511) / 512;
    uint4 v[NI];
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int i = tid + it * 512;
      const int n = i / CH, k = i % CH;
      if (i < TOT) v[it] = *reinterpret_cast<const uint4*>(w1 + (long)gch(n) * C + 8 * k);
    }
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int i = tid + it * 512;
      const int n = i / CH, k = i % CH;
      if (i < TOT) *reinterpret_cast<uint4*>(smem + n * WROW + ((k ^ (n & 15)) << 4)) = v[it];
    }
  }
  float bias[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bias[j] = p.b1[gch(j * 32 + r)];
  // the depthwise phase's thread = (gate quad qg, column x, row group rg); its taps and biases are loaded here, their
  // latency under the GEMM
  constexpr int NQG = GS / 4, RG = 512 / (NQG * S), RPG = S / RG;
  static_assert(NQG * S * RG == 512 && RPG * RG == S, "depthwise thread map");
  const int qg = tid % NQG, x = (tid / NQG) % S, rg = tid / (NQG * S);
  const int la = 4 * qg, lb = GS + 4 * qg;       // frame channels
  const int gca = cbase + 4 * qg, gcb = C + gca;  // conv channels
  f2v wa[9][2], wb[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      wa[t][hh] = f2v{p.wdw[(gca + 2 * hh) * 9 + t], p.wdw[(gca + 2 * hh + 1) * 9 + t]};
      wb[t][hh] = f2v{p.wdw[(gcb + 2 * hh) * 9 + t], p.wdw[(gcb + 2 * hh + 1) * 9 + t]};
    }
  const float4 ba = ld4(p.bdw + gca), bb = ld4(p.bdw + gcb);
  lds_barrier();

  // ---- phase 1: t1 tile = n1 rows . W1 slice^T (K ascending in steps of 16: the tiled GEMM's MFMA order)
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
#pragma unroll
  for (int t = 0; t < NST; ++t) {
    // retire stage t (the stages issued after it stay in flight); the MFMAs of stage t - 1 consumed its slot's reads
    if (NSTG >= 4 && t + 2 < NST) wait_vm<2 * PIECES>();
    else if (t + 1 < NST) wait_vm<PIECES>();
    else wait_vm<0>();
    if (t + NSTG - 1 < NST) issue(t + NSTG - 1);
    const unsigned char* st = ring + (t % NSTG) * STG;
#pragma unroll
    for (int j = 0; j < KC / 16; ++j) {
      const int s = t * (KC / 16) + j;
      vec_t<H, 8> bf[TN], a[TM];
#pragma unroll
      for (int jj = 0; jj < TN; ++jj) {
        const int n = jj * 32 + r;
        bf[jj] = *reinterpret_cast<const vec_t<H, 8>*>(smem + n * WROW + (((2 * s + h) ^ (n & 15)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = i * 32 + r;
        a[i] = *reinterpret_cast<const vec_t<H, 8>*>(st + row * RB + (((2 * j + h) ^ swz(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < TN; ++jj) acc[i][jj] = mfma32x32x16(a[i], bf[jj], acc[i][jj]);
    }
  }
  lds_barrier();  // every wave is done with the weight slice: the frame aliases it

  // ---- phase 2: t1 = H(acc + b1) into the zero-bordered frame [S + 2][S + 2][NCH]
  H* fr = reinterpret_cast<H*>(smem);
  {
    constexpr int BORDER = 4 * S + 4, CPC = NCH * 2 / 16, TOTB = BORDER * CPC;  // border cells, 16-B chunks per cell
    for (int i = tid; i < TOTB; i += 512) {
      const int cell = i / CPC, k = i % CPC;
      int py, px;
      if (cell < FW) py = 0, px = cell;                                  // top row
      else if (cell < 2 * FW) py = FW - 1, px = cell - FW;               // bottom row
      else if (cell < 2 * FW + S) py = 1 + (cell - 2 * FW), px = 0;      // left column
      else py = 1 + (cell - 2 * FW - S), px = FW - 1;                    // right column
      *reinterpret_cast<uint4*>(fr + (py * FW + px) * NCH + 8 * k) = make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int m = wave * 32 * TM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        const int py = m / S, px = m % S;
        fr[((py + 1) * FW + px + 1) * NCH + j * 32 + r] = (H)(acc[i][j][e] + bias[j]);
      }
  lds_barrier();

  // ---- phase 3a: t1 to memory (16-byte chunks; the slice's two channel runs per pixel)
  {
    constexpr int CPR = GS * 2 / 16, TOT = HW * 2 * CPR, NI = TOT / 512;
    static_assert(TOT % 512 == 0, "t1 store split");
    H* t1 = reinterpret_cast<H*>(p.t1) + (long)b * HW * 2 * C;
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int i = tid + it * 512;
      const int m = i / (2 * CPR), rk = i % (2 * CPR), run = rk / CPR, k = rk % CPR;
      const int py = m / S, px = m % S;
      const uint4 v = *reinterpret_cast<const uint4*>(fr + ((py + 1) * FW + px + 1) * NCH + run * GS + 8 * k);
      *reinterpret_cast<uint4*>(t1 + (long)m * 2 * C + run * C + cbase + 8 * k) = v;
    }
  }
  // ---- phase 3b: depthwise 3x3 + SimpleGate + pool
  const int r0 = rg * RPG;  // first image row of the group; frame row r0 = image row r0 - 1
  f2v xa[3][3][2], xb[3][3][2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    ldq2(fr + ((r0 + 0) * FW + x + j) * NCH + la, xa[1][j][0], xa[1][j][1]);
    ldq2(fr + ((r0 + 1) * FW + x + j) * NCH + la, xa[2][j][0], xa[2][j][1]);
    ldq2(fr + ((r0 + 0) * FW + x + j) * NCH + lb, xb[1][j][0], xb[1][j][1]);
    ldq2(fr + ((r0 + 1) * FW + x + j) * NCH + lb, xb[2][j][0], xb[2][j][1]);
  }
  H* t2p = p.t2 ? reinterpret_cast<H*>(p.t2) + ((long)b * HW + (long)r0 * S + x) * 2 * C : nullptr;
  H* gp = reinterpret_cast<H*>(p.g) + ((long)b * HW + (long)r0 * S + x) * C;
  float4 pacc = f4(0.f);
#pragma unroll
  for (int rr = 0; rr < RPG; ++rr) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        xa[0][j][hh] = xa[1][j][hh]; xa[1][j][hh] = xa[2][j][hh];
        xb[0][j][hh] = xb[1][j][hh]; xb[1][j][hh] = xb[2][j][hh];
      }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      ldq2(fr + ((r0 + rr + 2) * FW + x + j) * NCH + la, xa[2][j][0], xa[2][j][1]);
      ldq2(fr + ((r0 + rr + 2) * FW + x + j) * NCH + lb, xb[2][j][0], xb[2][j][1]);
    }
    f2v a2[2] = {f2v{ba.x, ba.y}, f2v{ba.z, ba.w}}, b2[2] = {f2v{bb.x, bb.y}, f2v{bb.z, bb.w}};
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        a2[hh] = __builtin_elementwise_fma(wa[t][hh], xa[t / 3][t % 3][hh], a2[hh]);
        b2[hh] = __builtin_elementwise_fma(wb[t][hh], xb[t / 3][t % 3][hh], b2[hh]);
      }
    const float4 aa = make_float4(a2[0].x, a2[0].y, a2[1].x, a2[1].y);
    const float4 ab = make_float4(b2[0].x, b2[0].y, b2[1].x, b2[1].y);
    if (t2p) {
      H* q2 = t2p + (long)rr * S * 2 * C;
      stq(q2 + gca, aa);
      stq(q2 + gcb, ab);
    }
    float4 gv = aa * ab;
    // the fp32 product is what is rounded to the storage type (the SimpleGate convention of every kernel)
    asm volatile("" : "+v"(gv.x), "+v"(gv.y), "+v"(gv.z), "+v"(gv.w));
    stq(gp + (long)rr * S * C + gca, gv);
    pacc += gv;
  }
  // ---- the slice's pool sums: the lanes of a gate quad in the wave (lane bits >= log2 NQG), then the 8 waves, in
  // a fixed order
#pragma unroll
  for (int o = NQG; o < 64; o <<= 1) {
    pacc.x += __shfl_xor(pacc.x, o, 64); pacc.y += __shfl_xor(pacc.y, o, 64);
    pacc.z += __shfl_xor(pacc.z, o, 64); pacc.w += __shfl_xor(pacc.w, o, 64);
  }
  lds_barrier();  // every depthwise read of the frame is done: reuse it
  float4* red = reinterpret_cast<float4*>(smem);
  if (lane < NQG) red[wave * NQG + lane] = pacc;
  lds_barrier();
  if (tid < GS) {
    const int q = tid >> 2, cpt = tid & 3;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) sum += get(red[w * NQG + q], cpt);
    p.pool[(long)b * C + cbase + tid] = sum;
  }
}

}  // namespace
}  // namespace nbp

using namespace nbp;

extern "C" {

// 1: the whole-image conv1 -> depthwise -> SimpleGate -> pool launch serves this block shape (16-bit storage; the
// 16 x 16 level at C 512).  The 32 x 32 level at C 256 (the same kernel, c1_dw_sg_pool_img<H, 256, 32, 32>) measured
// 50.4 us against 27.6 us for the two launches (scripts/c1dw_micro.py): a workgroup streams 1024 pixel rows per
// channel slice, through 32-byte ring rows (each line fetched four times), and its depthwise phase is twice the
// middle level's -- not served.
int nbp_c1dw_supported(int h, int w, int C, int dtype) {
  if (dtype != 1 && dtype != 2) return 0;
  return h == 16 && w == 16 && C == 512 ? 1 : 0;
}

int nbp_c1_dw_sg_pool(const void* n1, const void* w1, const float* b1, const float* wdw, const float* bdw, void* t1,
                      void* t2, void* g, float* pool, int B, int h, int w, int C, int dtype, nbp_stream_t s) {
  NBP_REQUIRE(n1 && w1 && b1 && wdw && bdw && t1 && g && pool && B > 0, "nbp_c1_dw_sg_pool: null pointer");
  NBP_REQUIRE(nbp_c1dw_supported(h, w, C, dtype), "nbp_c1_dw_sg_pool: unsupported shape (H %d W %d C %d dtype %d)",
              h, w, C, dtype);
  C1DwP p{n1, w1, b1, wdw, bdw, t1, t2, g, pool, B};
  NBP_DISPATCH_H(dtype, { c1_dw_sg_pool_img<H, 512, 16, 64><<<B * 16, 512, 0, S(s)>>>(p); });
  return check_launch("c1_dw_sg_pool");
}

}  // extern "C"
