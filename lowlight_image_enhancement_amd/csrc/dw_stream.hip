// SCA + SimpleGate + depthwise 3x3 backward over the stored tape, by row streaming (VERDICT r4 item 5;
// NAFNet_arch.py:60-67: dh -> dg = dh a + ds / HW (SCA), dt2 = (dg t2[C:], dg t2[:C]) (SimpleGate), dt1 = the depthwise
// conv's input gradient, dW / db its weight / bias gradients).  The replacement of dw_bwd_tiled (dwconv.hip) for the
// 16-bit modes (C % 16 == 0).
//
// dw_bwd_tiled stages one 18 x 34-pixel tile (t1 and the dt2 it forms from dh / t2) per workgroup in 78 KB of LDS, then
// walks the tile's 16 rows: two workgroups per CU, each loading before computing, so the loads and the arithmetic of a
// CU barely overlap.  Here a workgroup walks a strip of SH rows x 32 columns x one slice of 16 gate channels (+ their 16
// SimpleGate partners) with the same thread map and arithmetic (thread = channel quad q x column x; rolling 3 x 3
// register windows of dt2 and t1; per row dt1 by taps 0..8 from zero, dW / db accumulated), but the rows stream:
//   * each thread stages its own pixel of row k (dh and the partner half of t2 -> dt2 = round(dg t2'), and its t1 quad)
//     into a 4-slot 16-bit LDS ring (17 KB; 16 threads also stage the two halo columns), the row's loads issued U = 3
//     rows ahead into a register ring with static slots;
//   * per output row r: read ring row r + 2 (3 pixels of dt2 and t1; staged before the last barrier), roll the
//     windows, store dt1 row r, accumulate dW / db; stage row r + 3 into the slot of row r - 1 (last read at row r - 3,
//     or never), then one barrier.
// Bytes per pixel and slice: those of the stored-tape backward (dh C + t2 2C + t1 2C in, dt1 2C out) + 2 halo rows
// per strip (SH 64 / 32 / 16 / 8: the tallest giving >= 512 workgroups) and 2 halo columns per 32.
//
// Bitwise contract: dt2 = round(fma(dh, a, ds / HW) * t2[partner]) (0 outside the image), dt1 = taps 0..8 from zero by
// fused multiply-add, as dw_bwd_tiled (tests/test_gpu_dw_stream.py: dt1 bitwise); dW / db are per-strip partial sums
// (float64-bounded in the test).
#include "rowring.h"

namespace nbp {

struct DwStreamP {
  const void* dh;    // [M][C]
  const float* a;    // [B][C]
  const float* ds;   // [B][C]
  const void* t2;    // [M][2C]
  const void* t1;    // [M][2C]
  const float* wdw;  // [2C][9]
  void* dt1;         // [M][2C] out
  float* slab_w;     // [B * strips][2C][9] out
  float* slab_b;     // [B * strips][2C] out
  int B, H, W, C, SH, strips_x, strips;
  float inv_hw;
};

namespace {

constexpr int DS_TW = 32;  // strip width

template <typename T, int U>
__global__ __launch_bounds__(256, 2) void dw_bwd_stream(DwStreamP p) {
  constexpr int TW = DS_TW, LW = TW + 2;  // ring pixel px = image column x0 - 1 + px
  constexpr int CSL = 32, HS = 16, NQ = 8;  // conv channels per slice (16 gate + 16 partners), quads
  __shared__ __attribute__((aligned(16))) T sg[8 * LW * CSL];  // dt2 rows
  __shared__ __attribute__((aligned(16))) T sx[8 * LW * CSL];  // t1 rows
  const int tid = threadIdx.x;
  const int C = p.C, C2 = 2 * C, NSL = C / HS;
  const int u = xcd_remap(blockIdx.x, gridDim.x);  // the slices of one strip, then neighbouring strips, on one XCD
  const int slice = u % NSL, strip = (u / NSL) % p.strips, b = u / (NSL * p.strips);
  const int SH = p.SH;
  const int y0 = (strip / p.strips_x) * SH, x0 = (strip % p.strips_x) * TW;
  const int H = p.H, W = p.W;
  const long img = (long)b * H * W, M = (long)p.B * H * W;
  const __amdgpu_buffer_rsrc_t rh = rsrc(p.dh, M * C * 2), r2 = rsrc(p.t2, M * C * 4), r1 = rsrc(p.t1, M * C * 4),
                               ro = rsrc(p.dt1, M * C * 4);
  const int cbase = slice * HS;
  const int q = tid % NQ, x = tid / NQ;
  const int lc = 4 * q;                                               // slice-local channel of the quad
  const int gc = lc < HS ? cbase + lc : C + cbase + (lc - HS);        // its conv channel
  const int hc = lc < HS ? cbase + lc : cbase + (lc - HS);            // the gate channel (dh, a, ds)
  const int oc = lc < HS ? C + hc : hc;                               // the SimpleGate partner's t2 channel
  f2v wk[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) wk[t][h2] = f2v{p.wdw[(gc + 2 * h2) * 9 + t], p.wdw[(gc + 2 * h2 + 1) * 9 + t]};
  const float4 ak = ld4(p.a + (long)b * C + hc);
  const float4 sk = ld4(p.ds + (long)b * C + hc) * f4(p.inv_hw);
  // the staging pixel of this thread: ring pixel x + 1; threads of column 0 / 31 also stage ring pixel 0 / LW - 1
  const bool halo = x == 0 || x == TW - 1;
  const int hpx = x == 0 ? 0 : LW - 1;
  auto ok = [&](int yy, int gx) { return yy >= 0 && yy < H && gx >= 0 && gx < W; };
  auto off = [&](int yy, int gx, bool on, int pxb, int ch) {
    return on && ok(yy, gx) ? (int)((img + (long)yy * W + gx) * pxb) + 2 * ch : OOB;
  };
  vec_t<T, 4> rd[U], rt[U], rx[U], hd[U], ht[U], hx[U];  // ring row k's loads in slot k % U
  auto load = [&](int S, int k) {
    const int yy = y0 - 1 + k, gx = x0 + x, hx_ = x0 - 1 + hpx;
    rd[S] = bload4<T>(rh, off(yy, gx, true, 2 * C, hc));
    rt[S] = bload4<T>(r2, off(yy, gx, true, 4 * C, oc));
    rx[S] = bload4<T>(r1, off(yy, gx, true, 4 * C, gc));
    hd[S] = bload4<T>(rh, off(yy, hx_, halo, 2 * C, hc));
    ht[S] = bload4<T>(r2, off(yy, hx_, halo, 4 * C, oc));
    hx[S] = bload4<T>(r1, off(yy, hx_, halo, 4 * C, gc));
  };
  // dt2 of one pixel quad (0 outside the image) and its t1 quad into ring row k
  auto stage_px = [&](int k, int px, const vec_t<T, 4>& d, const vec_t<T, 4>& t2o, const vec_t<T, 4>& t1q) {
    const int yy = y0 - 1 + k, gx = x0 - 1 + px;
    const bool inside = ok(yy, gx);
    const float av[4] = {ak.x, ak.y, ak.z, ak.w}, sv[4] = {sk.x, sk.y, sk.z, sk.w};
    vec_t<T, 4> o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float dg = fmaf((float)d[e], av[e], sv[e]);
      float pr = dg * (float)t2o[e];
      asm volatile("" : "+v"(pr));  // the fp32 product is what is rounded (every SimpleGate kernel's convention)
      o[e] = inside ? (T)pr : (T)0.f;
    }
    const int slot = (k & 7) * LW * CSL + px * CSL + lc;
    *reinterpret_cast<vec_t<T, 4>*>(sg + slot) = o;
    *reinterpret_cast<vec_t<T, 4>*>(sx + slot) = t1q;
  };
  auto stage = [&](int S, int k) {
    stage_px(k, x + 1, rd[S], rt[S], rx[S]);
    if (halo) stage_px(k, hpx, hd[S], ht[S], hx[S]);
  };
  // this thread's 3-pixel window of ring row k: dt2 and t1 as packed fp32 pairs
  auto read3 = [&](int k, f2v (*g)[2], f2v (*xx)[2]) {
    const int base = (k & 7) * LW * CSL;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      ldq2(sg + base + (x + j) * CSL + lc, g[j][0], g[j][1]);
      ldq2(sx + base + (x + j) * CSL + lc, xx[j][0], xx[j][1]);
    }
  };
  // prologue: ring rows 0..3 staged, rows 4 .. U + 3 in flight
#pragma unroll
  for (int k = 0; k < 4; ++k) load(k % U, k);
#pragma unroll
  for (int k = 0; k < 4; ++k) stage(k % U, k);
#pragma unroll
  for (int k = 4; k < 4 + U; ++k) load(k % U, k);
  lds_barrier();
  f2v gw[3][3][2], xw[3][3][2];
  read3(0, gw[1], xw[1]);
  read3(1, gw[2], xw[2]);
  f2v aw[9][2], ab[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
#pragma unroll
  for (int t = 0; t < 9; ++t) aw[t][0] = aw[t][1] = f2v{0.f, 0.f};
  const int gx_own = x0 + x;

  // row r: read ring row r + 2, roll, dt1 row r + dW; stage ring row r + 3 (register slot (r + 3) % U = r % U, ring
  // slot (r + 3) & 3)
  auto row = [&](auto j_c, int r) {
    constexpr int J = decltype(j_c)::value;  // r % 4: the register slot of ring row r + 4; a barrier after odd rows
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        gw[0][j][h2] = gw[1][j][h2]; gw[1][j][h2] = gw[2][j][h2];
        xw[0][j][h2] = xw[1][j][h2]; xw[1][j][h2] = xw[2][j][h2];
      }
    read3(r + 2, gw[2], xw[2]);
    f2v acc[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
#pragma unroll
    for (int dh = -1; dh <= 1; ++dh)
#pragma unroll
      for (int dw = -1; dw <= 1; ++dw) {
        const int t = (dh + 1) * 3 + (dw + 1);
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          acc[h2] = __builtin_elementwise_fma(wk[t][h2], gw[1 - dh][1 - dw][h2], acc[h2]);
          aw[t][h2] = __builtin_elementwise_fma(gw[1][1][h2], xw[1 + dh][1 + dw][h2], aw[t][h2]);
        }
      }
    ab[0] += gw[1][1][0];
    ab[1] += gw[1][1][1];
    const int yr = y0 + r;
    bstore4<T>(ro, r < SH && yr < H && gx_own < W ? (int)((img + (long)yr * W + gx_own) * (4 * C)) + 2 * gc : OOB,
               make_float4(acc[0].x, acc[0].y, acc[1].x, acc[1].y));
    stage(J, r + 4);
    load(J, r + 4 + U);
    if constexpr (J & 1) lds_barrier();
  };

  static_assert(U == 4, "ring depth: the row loop is unrolled by 4");
  int r = 0;
#pragma unroll 1
  for (; r + 4 <= SH; r += 4) {
    row(IC<0>{}, r);
    row(IC<1>{}, r + 1);
    row(IC<2>{}, r + 2);
    row(IC<3>{}, r + 3);
  }
  if (r < SH) row(IC<0>{}, r);
  if (r + 1 < SH) row(IC<1>{}, r + 1);
  if (r + 2 < SH) row(IC<2>{}, r + 2);
  lds_barrier();  // (an even row count ends without one)
  // ---- reduce the 40 partials over the strip's columns (lane bits 3..5: reduce-scatter), then across the 4 waves
  float v[40];
#pragma unroll
  for (int t = 0; t < 10; ++t) {
    const f2v a0 = t < 9 ? aw[t][0] : ab[0], a1 = t < 9 ? aw[t][1] : ab[1];
    v[4 * t] = a0.x; v[4 * t + 1] = a0.y; v[4 * t + 2] = a1.x; v[4 * t + 3] = a1.y;
  }
  const int lane = tid & 63, wave = tid >> 6;
  float v2[20], v3[10], v4[5];
  const bool b3 = lane & 8, b4 = lane & 16, b5 = lane & 32;
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
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const float snd = b5 ? v3[j] : v3[j + 5], keep = b5 ? v3[j + 5] : v3[j];
    v4[j] = keep + __shfl_xor(snd, 32, 64);
  }
  float* red = reinterpret_cast<float*>(sg);  // the rings are dead (the last row ended with a barrier)
  const int e0 = (b3 ? 20 : 0) + (b4 ? 10 : 0) + (b5 ? 5 : 0);
#pragma unroll
  for (int j = 0; j < 5; ++j) red[(wave * NQ + (lane & 7)) * 40 + e0 + j] = v4[j];
  lds_barrier();
  const long row_id = (long)b * p.strips + strip;
  for (int i = tid; i < NQ * 40; i += 256) {
    const int qq = i / 40, e = i % 40, t = e >> 2, j = e & 3;
    const float s = ((red[(0 * NQ + qq) * 40 + e] + red[(1 * NQ + qq) * 40 + e]) + red[(2 * NQ + qq) * 40 + e]) +
                    red[(3 * NQ + qq) * 40 + e];
    const int l = 4 * qq + j;
    const int ch = l < HS ? cbase + l : C + cbase + (l - HS);
    if (t < 9) p.slab_w[(row_id * C2 + ch) * 9 + t] = s;
    else p.slab_b[row_id * C2 + ch] = s;
  }
}

}  // namespace

// strip height: the tallest of 64 / 32 / 16 / 8 rows whose grid still gives >= 512 workgroups (2 per CU)
int dw_stream_sh(int B, int H, int W, int C) {
  int sh = 64;
  while (sh > 8 && (long)B * cdiv(H, sh) * cdiv(W, DS_TW) * (C / 16) < 512) sh /= 2;
  return sh;
}
long dw_stream_rows(int B, int H, int W, int C) {
  const int sh = dw_stream_sh(B, H, W, C);
  return (long)B * cdiv(H, sh) * cdiv(W, DS_TW);
}
bool dw_stream_ok(int B, int H, int W, int C, int dtype) {
  return (dtype == 1 || dtype == 2) && C % 16 == 0 && C > 0 && (long)B * H * W * C * 4 < (1L << 31);
}

// the launch + its slab reductions; ws >= dw_stream_rows * 2C * 10 floats
int launch_dw_stream(const void* dh, const float* a, const float* ds, const void* t2, const void* t1, const float* wdw,
                     void* dt1, float* dwdw, float* dbdw, float* ws, int B, int H, int W, int C, int dtype,
                     nbp_stream_t s) {
  NBP_REQUIRE(dw_stream_ok(B, H, W, C, dtype), "dw_bwd_stream: unsupported shape (B %d H %d W %d C %d dtype %d)", B, H,
              W, C, dtype);
  DwStreamP p{};
  p.dh = dh; p.a = a; p.ds = ds; p.t2 = t2; p.t1 = t1; p.wdw = wdw; p.dt1 = dt1;
  p.B = B; p.H = H; p.W = W; p.C = C; p.SH = dw_stream_sh(B, H, W, C);
  p.strips_x = cdiv(W, DS_TW); p.strips = cdiv(H, p.SH) * p.strips_x;
  p.inv_hw = 1.f / (float)((long)H * W);
  const long nrow = (long)B * p.strips;
  p.slab_w = ws;
  p.slab_b = ws + nrow * 2 * C * 9;
  const long nblk = nrow * (C / 16);
  NBP_REQUIRE(nblk < (1L << 31), "dw_bwd_stream: grid too large");
  NBP_DISPATCH_H(dtype, { dw_bwd_stream<H, 4><<<nblk, 256, 0, S(s)>>>(p); });
  int rc = check_launch("dw_bwd_stream");
  if (rc) return rc;
  rc = nbp_reduce_slab(p.slab_w, (int)nrow, 2L * C * 9, dwdw, s);
  if (rc) return rc;
  return nbp_reduce_slab(p.slab_b, (int)nrow, 2L * C, dbdw, s);
}

}  // namespace nbp
