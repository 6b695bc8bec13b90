// MI355X (gfx950) turbo-decoder kernels: bit-exact re-implementations of the srsLTE 18.09
// max-log-MAP constituent decoders (paths relative to /root/reference/lib):
//   * windowed decoders  include/srslte/phy/fec/turbodecoder_win.h (AVX16: 16 sub-blocks,
//     SSE16: 8 sub-blocks + output >>1), saturating int16
//   * SSE non-window     src/phy/fec/turbodecoder_sse.c (halved branch metrics, wrapping int16)
//   * generic            src/phy/fec/turbodecoder_gen.c (wrapping int16)
// and the half-iteration glue of include/srslte/phy/fec/turbodecoder_iter.h:283-357.
//
// Data layout (HBM): code blocks are processed in PAIRS. Every per-CB int16 array is stored
// pair-interleaved as short2 [npairs][K] — element j of CB 2p sits in .x, of CB 2p+1 in .y —
// so one packed VALU op (v_pk_add_i16 clamp, v_pk_max_i16) advances both chains of a lane.
// Inside a code block the index j is the reference's sub-block (SB) index: j = k*NB + d holds
// natural position d*(K/NB) + k (rm_turbo.c:239-264), so the 16 (or 8) chains of one pair that
// run in lockstep at step k touch NB consecutive short2, and, because QPP interleavers are
// contention-free for every window length dividing K, the interleaver gathers of one step also
// hit NB consecutive elements.
//
// Windowed decoder mapping: one lane = one sub-block chain of one CB pair; a 64-lane wave
// carries 64/NB pairs. The backward (beta) pass keeps only every W-th state metric (plus the
// one at L) in a coalesced global checkpoint buffer; the forward (alpha) pass recomputes the W
// betas of each segment from its checkpoint into registers (exact: integer recursion) and
// emits the LLRs. This avoids streaming 16 B/bit/half-iteration of beta through HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tdec_kernels.h"

namespace srsgpu {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef short s4 __attribute__((ext_vector_type(4)));

#define TD_INF 10000  // turbodecoder_win.h:63 / _sse.c:51 / _gen.c:41
#define TD_OVERLAP 40 // turbodecoder_win.h:59 win_overlap_len

__device__ __forceinline__ s2 sadd(s2 a, s2 b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ s2 ssub(s2 a, s2 b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ s2 smax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
// wrapping int16 arithmetic on packed halves (v_pk_add_u16 / v_pk_sub_u16)
__device__ __forceinline__ s2 wadd(s2 a, s2 b) {
  typedef unsigned short u2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(s2, __builtin_bit_cast(u2, a) + __builtin_bit_cast(u2, b));
}
__device__ __forceinline__ s2 wsub(s2 a, s2 b) {
  typedef unsigned short u2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(s2, __builtin_bit_cast(u2, a) - __builtin_bit_cast(u2, b));
}
__device__ __forceinline__ s2 splat(short v) { return s2{v, v}; }

struct St8 {
  s2 s[8];
};

// ------------------------------------------------------------------ windowed steps ----

// turbodecoder_win.h:244-261 (16-bit): subtract state 0 every 2 steps, never at k == 0
__device__ __forceinline__ void win_norm(int k, St8 &o) {
  if ((k & 1) == 0 && k != 0) {
    s2 z = o.s[0];
#pragma unroll
    for (int i = 0; i < 8; i++) o.s[i] = ssub(o.s[i], z);
  }
}

// turbodecoder_win.h:395-418 backward step (saturating)
__device__ __forceinline__ void win_beta_step(St8 &o, s2 x, s2 y) {
  s2 xy = sadd(x, y);
  s2 b0 = o.s[0], b1 = o.s[1], b2 = o.s[2], b3 = o.s[3];
  s2 b4 = o.s[4], b5 = o.s[5], b6 = o.s[6], b7 = o.s[7];
  o.s[0] = smax(sadd(b4, xy), b0);
  o.s[1] = smax(b4, sadd(b0, xy));
  o.s[2] = smax(sadd(b5, y), sadd(b1, x));
  o.s[3] = smax(sadd(b5, x), sadd(b1, y));
  o.s[4] = smax(sadd(b6, x), sadd(b2, y));
  o.s[5] = smax(sadd(b6, y), sadd(b2, x));
  o.s[6] = smax(b7, sadd(b3, xy));
  o.s[7] = smax(sadd(b7, xy), b3);
}

// turbodecoder_win.h:521-539 forward branch sums (mb: input bit 0, nw: input bit 1)
__device__ __forceinline__ void win_alpha_branches(const St8 &o, s2 x, s2 y, s2 mb[8],
                                                   s2 nw[8]) {
  s2 xy = sadd(x, y);
  mb[0] = o.s[0];
  mb[1] = sadd(o.s[3], y);
  mb[2] = sadd(o.s[4], y);
  mb[3] = o.s[7];
  mb[4] = o.s[1];
  mb[5] = sadd(o.s[2], y);
  mb[6] = sadd(o.s[5], y);
  mb[7] = o.s[6];
  nw[0] = sadd(o.s[1], xy);
  nw[1] = sadd(o.s[2], x);
  nw[2] = sadd(o.s[5], x);
  nw[3] = sadd(o.s[6], xy);
  nw[4] = sadd(o.s[0], xy);
  nw[5] = sadd(o.s[3], x);
  nw[6] = sadd(o.s[4], x);
  nw[7] = sadd(o.s[7], xy);
}

__device__ __forceinline__ void win_alpha_step(St8 &o, s2 x, s2 y) {
  s2 mb[8], nw[8];
  win_alpha_branches(o, x, y, mb, nw);
#pragma unroll
  for (int i = 0; i < 8; i++) o.s[i] = smax(mb[i], nw[i]);
}

// turbodecoder_win.h:263-307: 3 tail steps with plain wrapping int16 adds
__device__ __forceinline__ void win_tail_trellis(const s2 *tail, int xoff, St8 &o) {
  o.s[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) o.s[i] = splat(-TD_INF);
#pragma unroll
  for (int j = 2; j >= 0; j--) {
    s2 x = tail[xoff + 2 * j], y = tail[xoff + 2 * j + 1], xy = wadd(x, y);
    s2 b0 = o.s[0], b1 = o.s[1], b2 = o.s[2], b3 = o.s[3];
    s2 b4 = o.s[4], b5 = o.s[5], b6 = o.s[6], b7 = o.s[7];
    o.s[0] = smax(wadd(b4, xy), b0);
    o.s[1] = smax(b4, wadd(b0, xy));
    o.s[2] = smax(wadd(b5, y), wadd(b1, x));
    o.s[3] = smax(wadd(b5, x), wadd(b1, y));
    o.s[4] = smax(wadd(b6, x), wadd(b2, y));
    o.s[5] = smax(wadd(b6, y), wadd(b2, x));
    o.s[6] = smax(b7, wadd(b3, xy));
    o.s[7] = smax(wadd(b7, xy), b3);
  }
}

__device__ __forceinline__ void st_fill(St8 &o, short v0, short v) {
  o.s[0] = splat(v0);
#pragma unroll
  for (int i = 1; i < 8; i++) o.s[i] = splat(v);
}

// checkpoint slot of stored-beta index k (k = L or a multiple of W)
template <int W>
__device__ __forceinline__ int ck_slot(int k) { return (k + W - 1) / W; }

__device__ __forceinline__ void ck_store(s4 *ck, size_t off, const St8 &o) {
  s4 a = {o.s[0].x, o.s[0].y, o.s[1].x, o.s[1].y};
  s4 b = {o.s[2].x, o.s[2].y, o.s[3].x, o.s[3].y};
  s4 c = {o.s[4].x, o.s[4].y, o.s[5].x, o.s[5].y};
  s4 d = {o.s[6].x, o.s[6].y, o.s[7].x, o.s[7].y};
  ck[off * 4 + 0] = a;
  ck[off * 4 + 1] = b;
  ck[off * 4 + 2] = c;
  ck[off * 4 + 3] = d;
}
__device__ __forceinline__ void ck_load(const s4 *ck, size_t off, St8 &o) {
  s4 a = ck[off * 4 + 0], b = ck[off * 4 + 1], c = ck[off * 4 + 2], d = ck[off * 4 + 3];
  o.s[0] = s2{a.x, a.y};
  o.s[1] = s2{a.z, a.w};
  o.s[2] = s2{b.x, b.y};
  o.s[3] = s2{b.z, b.w};
  o.s[4] = s2{c.x, c.y};
  o.s[5] = s2{c.z, c.w};
  o.s[6] = s2{d.x, d.y};
  o.s[7] = s2{d.z, d.w};
}

// One constituent MAP decoder run (turbodecoder_win.h:614-622) for every sub-block chain of
// every CB pair. xy: short4 [npairs][K] = (x.a, x.b, y.a, y.b) at SB index; tail: short2
// [npairs][12]; out: short2 [npairs][K]; ck: checkpoint scratch.
template <int NB, int DIV, int W>
__global__ __launch_bounds__(256) void k_win_dec(const s4 *__restrict__ xy,
                                                 const s2 *__restrict__ tail, int tail_xoff,
                                                 s2 *__restrict__ out, s4 *__restrict__ ck,
                                                 const uint8_t *__restrict__ pair_done, int K,
                                                 int npairs) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  const int pair = g / NB;
  const int d = g % NB;
  if (pair >= npairs) return;
  if (pair_done && pair_done[pair]) return;
  const int L = K / NB;
  const int nlanes = npairs * NB;
  const s4 *in = xy + (size_t)pair * K;
  s2 *o_out = out + (size_t)pair * K;
  const s2 *tl = tail + (size_t)pair * 12;

  // ---------------- beta ----------------
  St8 o;
  {
    // turbodecoder_win.h:376-384,386-433 (loop_len = 40): estimate the state at the start of
    // sub-block d+1 from all-unknown states; move_right (:333-366) hands it to sub-block d.
    st_fill(o, -TD_INF, -TD_INF);
    const int dn = d + 1 < NB ? d + 1 : d; // last lane: result replaced by the tail trellis
#pragma unroll 8
    for (int k = TD_OVERLAP - 1; k >= 0; k--) {
      s4 v = in[k * NB + dn];
      win_beta_step(o, s2{v.x, v.y}, s2{v.z, v.w});
      win_norm(k, o);
    }
    St8 t;
    win_tail_trellis(tl, tail_xoff, t); // :350-355 last sub-block starts from the tail
    if (d == NB - 1) o = t;
  }
  ck_store(ck, (size_t)ck_slot<W>(L) * nlanes + g, o); // :372-374 beta[L]
  for (int k = L - 1; k >= 0; k--) {
    s4 v = in[k * NB + d];
    win_beta_step(o, s2{v.x, v.y}, s2{v.z, v.w});
    if ((k % W) == 0 && k != 0) ck_store(ck, (size_t)(k / W) * nlanes + g, o); // pre-normalise
    win_norm(k, o);
  }

  // ---------------- alpha + LLR ----------------
  {
    // :501-506,512-584 (loop_len = 40) over the last 40 steps of sub-block d-1; move_left
    // (:469-495) hands the estimate to sub-block d; sub-block 0 starts in state 0 (:496-500).
    st_fill(o, -TD_INF, -TD_INF);
    const int dp = d > 0 ? d - 1 : 0;
#pragma unroll 8
    for (int k = 0; k < TD_OVERLAP; k++) {
      s4 v = in[(L - TD_OVERLAP + k) * NB + dp];
      win_alpha_step(o, s2{v.x, v.y}, s2{v.z, v.w});
      win_norm(k, o);
    }
    if (d == 0) st_fill(o, 0, -TD_INF);
  }
  for (int s0 = 0; s0 < L; s0 += W) {
    const int s1 = s0 + W < L ? s0 + W : L;
    const int n = s1 - s0;
    s2 xs[W], ys[W];
#pragma unroll
    for (int j = 0; j < W; j++) {
      if (j < n) {
        s4 v = in[(s0 + j) * NB + d];
        xs[j] = s2{v.x, v.y};
        ys[j] = s2{v.z, v.w};
      }
    }
    // betas stored at indices s0+1 .. s1 (bst[j] = stored beta[s0+1+j])
    St8 bst[W];
    St8 run;
    ck_load(ck, (size_t)ck_slot<W>(s1) * nlanes + g, run);
#pragma unroll
    for (int j = W - 1; j >= 0; j--) {
      if (j == n - 1) bst[j] = run;
    }
    if (s1 != L) win_norm(s1, run); // running state continues from the normalised value
#pragma unroll
    for (int j = W - 2; j >= 0; j--) {
      if (j <= n - 2) {
        win_beta_step(run, xs[j + 1], ys[j + 1]);
        bst[j] = run;
        win_norm(s0 + 1 + j, run);
      }
    }
#pragma unroll
    for (int j = 0; j < W; j++) {
      if (j < n) {
        s2 mb[8], nw[8];
        win_alpha_branches(o, xs[j], ys[j], mb, nw);
        s2 m0 = sadd(bst[j].s[0], mb[0]);
        s2 m1 = sadd(bst[j].s[0], nw[0]);
#pragma unroll
        for (int i = 1; i < 8; i++) {
          m0 = smax(m0, sadd(bst[j].s[i], mb[i]));
          m1 = smax(m1, sadd(bst[j].s[i], nw[i]));
        }
        s2 v = ssub(m1, m0);
        if (DIV) v = v >> 1; // :565-567 srai 1 (SSE16 window)
        o_out[(s0 + j) * NB + d] = v;
#pragma unroll
        for (int i = 0; i < 8; i++) o.s[i] = smax(mb[i], nw[i]);
        win_norm(s0 + j, o);
      }
    }
  }
}

// ------------------------------------------------------------------ SSE non-window ----
// turbodecoder_sse.c:97-407, one lane per CB pair, natural index. x/app/par come through
// the xy stream (x already contains app, wrapping, as tdec_sse_gamma :321-325 does) — the
// caller builds it with wrapping adds for this decoder. Tail gammas use C division.
// scratch: alpha (K+1)*8 short2 per pair.
__global__ __launch_bounds__(64) void k_sse_dec(const s4 *__restrict__ xy,
                                                const s2 *__restrict__ tail, int tail_xoff,
                                                s2 *__restrict__ out, s2 *__restrict__ scratch,
                                                const uint8_t *__restrict__ pair_done, int K,
                                                int npairs) {
  const int pair = blockIdx.x * blockDim.x + threadIdx.x;
  if (pair >= npairs) return;
  if (pair_done && pair_done[pair]) return;
  const s4 *in = xy + (size_t)pair * K;
  s2 *o_out = out + (size_t)pair * K;
  const s2 *tl = tail + (size_t)pair * 12;
  // alpha in scratch, lane-interleaved so that consecutive pairs are contiguous
  auto AL = [&](int k, int i) -> s2 & { return scratch[((size_t)k * 8 + i) * npairs + pair]; };
  s2 a[8];
  a[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) a[i] = splat(-TD_INF);
#pragma unroll
  for (int i = 0; i < 8; i++) AL(0, i) = a[i];
  for (int k = 0; k < K; k++) { // :211-297
    s4 v = in[k];
    s2 x = s2{v.x, v.y}, y = s2{v.z, v.w};
    s2 g1 = wadd(x, y) >> 1, g0 = wsub(x, y) >> 1;
    s2 n[8];
    n[0] = smax(wadd(a[1], g1), wsub(a[0], g1));
    n[1] = smax(wadd(a[2], g0), wsub(a[3], g0));
    n[2] = smax(wadd(a[5], g0), wsub(a[4], g0));
    n[3] = smax(wadd(a[6], g1), wsub(a[7], g1));
    n[4] = smax(wadd(a[0], g1), wsub(a[1], g1));
    n[5] = smax(wadd(a[3], g0), wsub(a[2], g0));
    n[6] = smax(wadd(a[4], g0), wsub(a[5], g0));
    n[7] = smax(wadd(a[7], g1), wsub(a[6], g1));
#pragma unroll
    for (int i = 0; i < 8; i++) {
      a[i] = n[i];
      AL(k + 1, i) = a[i];
    }
    if ((k & 3) == 3) {
      s2 z = a[0];
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = wsub(a[i], z);
    }
  }
  s2 b[8];
  b[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) b[i] = splat(-TD_INF);
  for (int k = K + 2; k >= 0; k--) { // :105-206
    s2 g0, g1;
    if (k >= K) { // :349-352 C division truncates toward zero
      s2 x = tl[tail_xoff + 2 * (k - K)], y = tl[tail_xoff + 2 * (k - K) + 1];
      g0 = s2{(short)(((int)x.x - y.x) / 2), (short)(((int)x.y - y.y) / 2)};
      g1 = s2{(short)(((int)x.x + y.x) / 2), (short)(((int)x.y + y.y) / 2)};
    } else {
      s4 v = in[k];
      s2 x = s2{v.x, v.y}, y = s2{v.z, v.w};
      g1 = wadd(x, y) >> 1;
      g0 = wsub(x, y) >> 1;
    }
    s2 bp[8] = {wadd(b[4], g1), wadd(b[0], g1), wadd(b[1], g0), wadd(b[5], g0),
                wadd(b[6], g0), wadd(b[2], g0), wadd(b[3], g1), wadd(b[7], g1)};
    s2 bn[8] = {wsub(b[0], g1), wsub(b[4], g1), wsub(b[5], g0), wsub(b[1], g0),
                wsub(b[2], g0), wsub(b[6], g0), wsub(b[7], g1), wsub(b[3], g1)};
#pragma unroll
    for (int i = 0; i < 8; i++) b[i] = smax(bp[i], bn[i]);
    if (k < K) {
      s2 mp = splat(-32768), mn = splat(-32768);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        s2 al = AL(k, i);
        mp = smax(mp, wadd(bp[i], al));
        mn = smax(mn, wadd(bn[i], al));
      }
      // hMax(bn) - hMax(bp) with hMax(v) = 0x7FFF - max(v) (minpos_epu16 trick)
      o_out[k] = wsub(wsub(splat(0x7FFF), mn), wsub(splat(0x7FFF), mp));
      if ((k & 3) == 0) {
        s2 z = b[0];
#pragma unroll
        for (int i = 0; i < 8; i++) b[i] = wsub(b[i], z);
      }
    }
  }
}

// ------------------------------------------------------------------ generic ----
// turbodecoder_gen.c:59-236, one lane per CB pair, natural index, wrapping int16.
// The xy stream carries x = syst (+) app with a wrapping add (gen.c:72-74,120-122 add app only
// for k < K, which is exactly the stream's range); tail x/y come from the tail array.
// scratch: beta (K+4)*8 short2 per pair.
__global__ __launch_bounds__(64) void k_gen_dec(const s4 *__restrict__ xy,
                                                const s2 *__restrict__ tail, int tail_xoff,
                                                s2 *__restrict__ out, s2 *__restrict__ scratch,
                                                const uint8_t *__restrict__ pair_done, int K,
                                                int npairs) {
  const int pair = blockIdx.x * blockDim.x + threadIdx.x;
  if (pair >= npairs) return;
  if (pair_done && pair_done[pair]) return;
  const s4 *in = xy + (size_t)pair * K;
  s2 *o_out = out + (size_t)pair * K;
  const s2 *tl = tail + (size_t)pair * 12;
  auto BE = [&](int k, int i) -> s2 & { return scratch[((size_t)k * 8 + i) * npairs + pair]; };
  const int end = K + 3;
  s2 o[8];
  o[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) o[i] = splat(-TD_INF);
  for (int k = end - 1; k >= 0; k--) {
    s2 x, y;
    if (k >= K) {
      x = tl[tail_xoff + 2 * (k - K)];
      y = tl[tail_xoff + 2 * (k - K) + 1];
    } else {
      s4 v = in[k];
      x = s2{v.x, v.y};
      y = s2{v.z, v.w};
    }
    s2 xy_ = wadd(x, y);
    s2 mb[8] = {wadd(o[4], xy_), o[4], wadd(o[5], y), wadd(o[5], x),
                wadd(o[6], x), wadd(o[6], y), o[7], wadd(o[7], xy_)};
    s2 nw[8] = {o[0], wadd(o[0], xy_), wadd(o[1], x), wadd(o[1], y),
                wadd(o[2], y), wadd(o[2], x), wadd(o[3], xy_), o[3]};
#pragma unroll
    for (int i = 0; i < 8; i++) {
      o[i] = smax(mb[i], nw[i]);
      BE(k, i) = o[i];
    }
    if ((k & 3) == 0 && k < K) {
      s2 z = o[0];
#pragma unroll
      for (int i = 0; i < 8; i++) o[i] = wsub(o[i], z);
    }
  }
  s2 a[8];
  a[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) a[i] = splat(-TD_INF);
  for (int k = 1; k < K + 1; k++) {
    s4 v = in[k - 1];
    s2 x = s2{v.x, v.y}, y = s2{v.z, v.w}, xy_ = wadd(x, y);
    s2 mb[8] = {a[0], wadd(a[3], y), wadd(a[4], y), a[7],
                a[1], wadd(a[2], y), wadd(a[5], y), a[6]};
    s2 nw[8] = {wadd(a[1], xy_), wadd(a[2], x), wadd(a[5], x), wadd(a[6], xy_),
                wadd(a[0], xy_), wadd(a[3], x), wadd(a[4], x), wadd(a[7], xy_)};
    s2 m0 = wadd(mb[0], BE(k, 0)), m1 = wadd(nw[0], BE(k, 0));
#pragma unroll
    for (int i = 1; i < 8; i++) {
      s2 be = BE(k, i);
      m0 = smax(m0, wadd(mb[i], be));
      m1 = smax(m1, wadd(nw[i], be));
    }
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = smax(mb[i], nw[i]);
    if ((k & 3) == 0) {
      s2 z = a[0];
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = wsub(a[i], z);
    }
    o_out[k - 1] = wsub(m1, m0);
  }
}

// ------------------------------------------------------------------ glue kernels ----

// Input load: user layout -> pair-interleaved syst/par0/par1 (SB index when NB > 1) + tails.
// Natural input: [s,p0,p1]*K + 12 tail (turbodecoder_gen.c:240-259, win.h:634-674);
// SB input: streams at s*(K+32), tails at 3*(K+32) (turbodecoder_iter.h:271-280).
__global__ void k_load(const int16_t *__restrict__ in, size_t in_stride, int sb_input, int K,
                       int NB, int ncb, s2 *__restrict__ S, s2 *__restrict__ P0,
                       s2 *__restrict__ P1, s2 *__restrict__ T) {
  const int npairs = (ncb + 1) / 2;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = K + 12;
  if (tid >= (size_t)npairs * per) return;
  const int pair = (int)(tid / per);
  const int j = (int)(tid % per);
  const int c0 = 2 * pair, c1 = c0 + 1 < ncb ? c0 + 1 : c0;
  const int16_t *a = in + (size_t)c0 * in_stride, *b = in + (size_t)c1 * in_stride;
  if (j < K) {
    // j is the destination index (SB index when NB > 1)
    int s, p0, p1;
    if (sb_input) {
      s = j;
      p0 = (K + 32) + j;
      p1 = 2 * (K + 32) + j;
    } else {
      int p = j;
      if (NB > 1) {
        const int L = K / NB;
        p = (j % NB) * L + j / NB; // SB index -> natural position
      }
      s = 3 * p;
      p0 = 3 * p + 1;
      p1 = 3 * p + 2;
    }
    S[(size_t)pair * K + j] = s2{a[s], b[s]};
    P0[(size_t)pair * K + j] = s2{a[p0], b[p0]};
    P1[(size_t)pair * K + j] = s2{a[p1], b[p1]};
  } else {
    const int t = j - K;
    const int base = sb_input ? 3 * (K + 32) : 3 * K;
    T[(size_t)pair * 12 + t] = s2{a[base + t], b[base + t]};
  }
}

// Even half-iteration prologue (turbodecoder_iter.h:315-324): app1 = deinterleave(ext2)
// - ext1 (wrapping) for n > 0, decoder input x = syst (+) app1.
// mode: 0 = saturating add (windowed), 1 = wrapping add (SSE/generic).
__global__ void k_prep_even(int n, int K, int npairs, const uint16_t *__restrict__ rev,
                            const s2 *__restrict__ S, const s2 *__restrict__ P0,
                            const s2 *__restrict__ X2, const s2 *__restrict__ E,
                            s2 *__restrict__ A, s4 *__restrict__ XY, int wrap_mode,
                            const uint8_t *__restrict__ pair_done) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (size_t)npairs * K) return;
  const int pair = (int)(tid / K);
  if (pair_done && pair_done[pair]) return;
  const int j = (int)(tid % K);
  const size_t base = (size_t)pair * K;
  s2 x = S[base + j];
  if (n > 0) {
    s2 app = wsub(X2[base + rev[j]], E[base + j]);
    A[base + j] = app;
    x = wrap_mode ? wadd(x, app) : sadd(app, x);
  }
  s2 y = P0[base + j];
  XY[base + j] = s4{x.x, x.y, y.x, y.y};
}

// Odd half-iteration prologue (turbodecoder_iter.h:327-333): ext1 -= app1 for n > 1, then
// app2 = interleave(ext1): app2[m] = ext1[fwd[m]]. E is double-buffered (Ein -> Eout).
__global__ void k_prep_odd(int n, int K, int npairs, const uint16_t *__restrict__ fwd,
                           const s2 *__restrict__ P1, const s2 *__restrict__ Ein,
                           const s2 *__restrict__ A, s2 *__restrict__ Eout,
                           s4 *__restrict__ XY, const uint8_t *__restrict__ pair_done) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (size_t)npairs * K) return;
  const int pair = (int)(tid / K);
  if (pair_done && pair_done[pair]) return;
  const int m = (int)(tid % K);
  const size_t base = (size_t)pair * K;
  const int f = fwd[m];
  s2 x;
  if (n > 1) {
    Eout[base + m] = wsub(Ein[base + m], A[base + m]);
    x = wsub(Ein[base + f], A[base + f]);
  } else {
    x = Ein[base + f];
  }
  s2 y = P1[base + m];
  XY[base + m] = s4{x.x, x.y, y.x, y.y};
}

// Hard decision after half-iteration n (turbodecoder.c:353-360 + decision_byte): bits from
// ext1 after DEC1 (n even) or from app1 = deinterleave(ext2) after DEC2 (n odd), natural order,
// MSB first. One thread per output byte. Skips CBs already finished (early stop).
__global__ void k_decide(int n, int K, int NB, int ncb, const uint16_t *__restrict__ rev,
                         const s2 *__restrict__ E, const s2 *__restrict__ X2,
                         uint8_t *__restrict__ outb, size_t out_stride,
                         const uint8_t *__restrict__ cb_done) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int nbytes = K / 8;
  if (tid >= (size_t)ncb * nbytes) return;
  const int cb = (int)(tid / nbytes);
  if (cb_done && cb_done[cb]) return;
  const int byte = (int)(tid % nbytes);
  const int pair = cb >> 1, half = cb & 1;
  const size_t base = (size_t)pair * K;
  const int L = K / NB;
  uint8_t r = 0;
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const int p = 8 * byte + b;
    const int j = NB > 1 ? (p % L) * NB + p / L : p;
    s2 v = (n & 1) ? X2[base + rev[j]] : E[base + j];
    short s = half ? v.y : v.x;
    if (s > 0) r |= (uint8_t)(0x80 >> b);
  }
  outb[(size_t)cb * out_stride + byte] = r;
}

// CRC check + early-stop bookkeeping (sch.c:361-391): one wave per CB; the byte-serial table
// CRC (crc.c:144-155) is split over 64 lanes as 64 partial CRCs combined by shifting through
// the zero-extension operator, done here by a simple sequential fold on lane 0 of the partial
// remainders (each partial is a table CRC of its 1/64 slice followed by zero bytes).
__global__ void k_crc_check(int n, int ncb, int nbytes_total, uint32_t poly,
                            const uint8_t *__restrict__ outb, size_t out_stride,
                            uint8_t *__restrict__ cb_done, uint8_t *__restrict__ cb_ok,
                            uint32_t *__restrict__ noi, int max_halfits) {
  __shared__ uint32_t table[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t crc = (uint32_t)i << 16;
    for (int j = 0; j < 8; j++) {
      uint32_t bit = crc & 0x800000u;
      crc <<= 1;
      if (bit) crc ^= poly;
    }
    table[i] = crc & 0xFFFFFFu;
  }
  __syncthreads();
  const int cb = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int lane = threadIdx.x & 63;
  if (cb >= ncb) return;
  if (cb_done[cb]) return;
  // lane 0 walks the bytes (K/8 <= 768 table steps); other lanes idle. Simple and exact.
  if (lane == 0) {
    const uint8_t *p = outb + (size_t)cb * out_stride;
    uint32_t crc = 0;
    for (int i = 0; i < nbytes_total; i++) {
      crc = ((crc << 8) ^ table[((crc >> 16) & 0xff) ^ p[i]]) & 0xFFFFFFu;
    }
    noi[cb] = (uint32_t)(n + 1);
    if (crc == 0) {
      cb_ok[cb] = 1;
      cb_done[cb] = 1;
    } else if (n + 1 >= max_halfits) {
      cb_done[cb] = 1;
    }
  }
}

// pair_done = cb_done[2p] && cb_done[2p+1]
__global__ void k_pair_done(int ncb, const uint8_t *__restrict__ cb_done,
                            uint8_t *__restrict__ pair_done) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  const int npairs = (ncb + 1) / 2;
  if (p >= npairs) return;
  const int c1 = 2 * p + 1 < ncb ? 2 * p + 1 : 2 * p;
  pair_done[p] = cb_done[2 * p] && cb_done[c1];
}

// ------------------------------------------------------------------ launchers ----

static inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

hipError_t launch_load(const int16_t *in, size_t in_stride, int sb_input, int K, int NB, int ncb,
                       void *S, void *P0, void *P1, void *T, hipStream_t st) {
  const int npairs = (ncb + 1) / 2;
  size_t n = (size_t)npairs * (K + 12);
  hipLaunchKernelGGL(k_load, dim3(nblk(n, 256)), dim3(256), 0, st, in, in_stride, sb_input, K, NB,
                     ncb, (s2 *)S, (s2 *)P0, (s2 *)P1, (s2 *)T);
  return hipGetLastError();
}

hipError_t launch_prep_even(int n, int K, int npairs, const uint16_t *rev, const void *S,
                            const void *P0, const void *X2, const void *E, void *A, void *XY,
                            int wrap_mode, const uint8_t *pair_done, hipStream_t st) {
  size_t tot = (size_t)npairs * K;
  hipLaunchKernelGGL(k_prep_even, dim3(nblk(tot, 256)), dim3(256), 0, st, n, K, npairs, rev,
                     (const s2 *)S, (const s2 *)P0, (const s2 *)X2, (const s2 *)E, (s2 *)A,
                     (s4 *)XY, wrap_mode, pair_done);
  return hipGetLastError();
}

hipError_t launch_prep_odd(int n, int K, int npairs, const uint16_t *fwd, const void *P1,
                           const void *Ein, const void *A, void *Eout, void *XY,
                           const uint8_t *pair_done, hipStream_t st) {
  size_t tot = (size_t)npairs * K;
  hipLaunchKernelGGL(k_prep_odd, dim3(nblk(tot, 256)), dim3(256), 0, st, n, K, npairs, fwd,
                     (const s2 *)P1, (const s2 *)Ein, (const s2 *)A, (s2 *)Eout, (s4 *)XY,
                     pair_done);
  return hipGetLastError();
}

size_t win_ck_bytes(int K, int NB, int npairs) {
  const int L = K / NB;
  const int W = TD_CK_W;
  size_t slots = (size_t)(L + W - 1) / W + 1;
  return slots * (size_t)npairs * NB * 8 * sizeof(s2);
}

hipError_t launch_win_dec(int NB, const void *XY, const void *T, int tail_xoff, void *out,
                          void *ck, const uint8_t *pair_done, int K, int npairs, hipStream_t st) {
  size_t lanes = (size_t)npairs * NB;
  dim3 grid(nblk(lanes, 256)), blk(256);
  if (NB == 16) {
    hipLaunchKernelGGL((k_win_dec<16, 0, TD_CK_W>), grid, blk, 0, st, (const s4 *)XY,
                       (const s2 *)T, tail_xoff, (s2 *)out, (s4 *)ck, pair_done, K, npairs);
  } else if (NB == 8) {
    hipLaunchKernelGGL((k_win_dec<8, 1, TD_CK_W>), grid, blk, 0, st, (const s4 *)XY,
                       (const s2 *)T, tail_xoff, (s2 *)out, (s4 *)ck, pair_done, K, npairs);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

size_t seq_scratch_bytes(int K, int npairs) { return (size_t)(K + 4) * 8 * npairs * sizeof(s2); }

hipError_t launch_sse_dec(const void *XY, const void *T, int tail_xoff, void *out, void *scratch,
                          const uint8_t *pair_done, int K, int npairs, hipStream_t st) {
  hipLaunchKernelGGL(k_sse_dec, dim3(nblk(npairs, 64)), dim3(64), 0, st, (const s4 *)XY,
                     (const s2 *)T, tail_xoff, (s2 *)out, (s2 *)scratch, pair_done, K, npairs);
  return hipGetLastError();
}

hipError_t launch_gen_dec(const void *XY, const void *T, int tail_xoff, void *out, void *scratch,
                          const uint8_t *pair_done, int K, int npairs, hipStream_t st) {
  hipLaunchKernelGGL(k_gen_dec, dim3(nblk(npairs, 64)), dim3(64), 0, st, (const s4 *)XY,
                     (const s2 *)T, tail_xoff, (s2 *)out, (s2 *)scratch, pair_done, K, npairs);
  return hipGetLastError();
}

hipError_t launch_decide(int n, int K, int NB, int ncb, const uint16_t *rev, const void *E,
                         const void *X2, uint8_t *outb, size_t out_stride, const uint8_t *cb_done,
                         hipStream_t st) {
  size_t tot = (size_t)ncb * (K / 8);
  hipLaunchKernelGGL(k_decide, dim3(nblk(tot, 256)), dim3(256), 0, st, n, K, NB, ncb, rev,
                     (const s2 *)E, (const s2 *)X2, outb, out_stride, cb_done);
  return hipGetLastError();
}

hipError_t launch_crc_check(int n, int ncb, int nbytes, uint32_t poly, const uint8_t *outb,
                            size_t out_stride, uint8_t *cb_done, uint8_t *cb_ok, uint32_t *noi,
                            int max_halfits, uint8_t *pair_done, hipStream_t st) {
  hipLaunchKernelGGL(k_crc_check, dim3(nblk(ncb, 4)), dim3(256), 0, st, n, ncb, nbytes, poly,
                     outb, out_stride, cb_done, cb_ok, noi, max_halfits);
  hipLaunchKernelGGL(k_pair_done, dim3(nblk((ncb + 1) / 2, 256)), dim3(256), 0, st, ncb, cb_done,
                     pair_done);
  return hipGetLastError();
}

} // namespace srsgpu
