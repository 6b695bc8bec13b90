// MI355X (gfx950) turbo-decoder kernels: bit-exact re-implementations of the srsLTE 18.09
// max-log-MAP constituent decoders (paths relative to /root/reference/lib):
//   * windowed decoders  include/srslte/phy/fec/turbodecoder_win.h (AVX16: 16 sub-blocks,
//     SSE16: 8 sub-blocks + output >>1), saturating int16
//   * SSE non-window     src/phy/fec/turbodecoder_sse.c (halved branch metrics, wrapping int16)
//   * generic            src/phy/fec/turbodecoder_gen.c (wrapping int16)
// with the half-iteration glue of include/srslte/phy/fec/turbodecoder_iter.h:283-357 fused into
// the decoder's output stage (no separate interleave/subtract passes).
//
// ---- Data layout in HBM ---------------------------------------------------------------------
// Code blocks are processed in PAIRS: every per-CB int16 array is stored pair-interleaved
// (element j of CB 2p in .x, of CB 2p+1 in .y) so one packed VALU op (v_pk_add_i16 clamp,
// v_pk_max_i16) advances both chains of a lane. Within a CB the index j is the reference's
// sub-block (SB) index: j = k*NB + d holds natural position d*(K/NB) + k (rm_turbo.c:239-264).
// The NB chains of one pair run in lockstep over k, so a step's loads touch NB consecutive
// elements; and since QPP interleavers are contention-free for every window length dividing K
// (pi(x + tW) = pi(x) mod W), the interleaver scatters of one step also land on NB consecutive
// elements (permuted) — every global access is a 64/128-byte coalesced group.
//   SP0[pair][K]  short4 (syst.a, syst.b, par0.a, par0.b)          static
//   X2 [pair][K]  short2  app2 (DEC2 input), rewritten by every DEC1 (dense, so the scattered
//                 DEC1 stores fill whole cache lines)
//   P1 [pair][K]  short2  par1                                      static (X2 + npairs*K)
//   A  [pair][K]  short2  app1 - ext1 ("a priori" of DEC1); the first DEC1 neither reads it nor
//                 needs it zeroed (MODE 2), DEC2 writes every element
//   T  [pair][12] short2  tail values as in the reference input (s,p0)x3 (app2,p1)x3
// Half-iteration n even (DEC1): x = syst (+) A, y = par0; the LLR L gives E' = L - A, scattered
//   to app2[rev[j]] (the reference's ext1 -= app1 and vec_lut interleave).
// n odd (DEC2): x = app2, y = par1; A[fwd[j]] = L - app2[j] (vec_lut deinterleave, app1 -= ext1).
// Hard decision after either: bit(p) = A + app2[rev] at j(p) > 0 (= ext1 after DEC1, app1 after
// DEC2, because both subtractions are exactly invertible modulo 2^16).
//
// ---- Groups ---------------------------------------------------------------------------------
// A job holds groups of code blocks (one K and decoder variant each, tdec_kernels.h). Every
// [pair][K] array above is the concatenation of the groups' arrays (group g from element elem0);
// pair-indexed arrays (T, pair_done) use the global pair index pair0 + p, CB-indexed ones (rows,
// outputs, flags) the caller's index cb0 + c. One launch per variant covers all its groups.
//
// ---- Windowed decoder mapping ---------------------------------------------------------------
// One lane = one sub-block chain of one CB pair, a 64-lane wave = 64/NB pairs (k_win_bidir).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "tdec_kernels.h"

namespace srsgpu {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef short s4 __attribute__((ext_vector_type(4)));

#define TD_INF 10000  // turbodecoder_win.h:63 / _sse.c:51 / _gen.c:41
#define TD_OVERLAP 40 // turbodecoder_win.h:59 win_overlap_len
#ifndef TD_BIDIR_CW
#define TD_BIDIR_CW 16 // checkpoint period of the bidirectional decoder (LDS checkpoints)
#endif

__device__ __forceinline__ s2 sadd(s2 a, s2 b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ s2 ssub(s2 a, s2 b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ s2 smax(s2 a, s2 b) { return __builtin_elementwise_max(a, b); }
// wrapping int16 arithmetic on packed halves (v_pk_add_u16 / v_pk_sub_u16)
typedef unsigned short u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s2 wadd(s2 a, s2 b) {
  return __builtin_bit_cast(s2, __builtin_bit_cast(u2, a) + __builtin_bit_cast(u2, b));
}
__device__ __forceinline__ s2 wsub(s2 a, s2 b) {
  return __builtin_bit_cast(s2, __builtin_bit_cast(u2, a) - __builtin_bit_cast(u2, b));
}
__device__ __forceinline__ s2 splat(short v) { return s2{v, v}; }
__device__ __forceinline__ s2 lo2(s4 v) { return s2{v.x, v.y}; }
__device__ __forceinline__ s2 hi2(s4 v) { return s2{v.z, v.w}; }

struct St8 {
  s2 s[8];
};

// Pointers read from a group descriptor are generic (flat) to the compiler; tables are global
// memory, and flat loads would count against both vmcnt and lgkmcnt. gptr() restores that.
template <typename T> using gptr_t = const T __attribute__((address_space(1))) *;
template <typename T> __device__ __forceinline__ gptr_t<T> gptr(const T *p) {
  return (gptr_t<T>)(const __attribute__((address_space(1))) void *)(uintptr_t)p;
}
template <typename T> using gmut_t = T __attribute__((address_space(1))) *;
template <typename T> __device__ __forceinline__ gmut_t<T> gmut(void *p) {
  return (gmut_t<T>)(__attribute__((address_space(1))) void *)(uintptr_t)p;
}

// group of workgroup b in a launch: the last group whose first workgroup (field F) is <= b
enum { GF_LOAD, GF_HALF, GF_PAIR };
template <int F>
__device__ __forceinline__ int grp_find(const TdGroup *__restrict__ g, int ng, int b) {
  int lo = 0, hi = ng - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int v = F == GF_LOAD ? g[mid].blk_load : F == GF_HALF ? g[mid].blk_half : g[mid].pair0;
    if (v <= b)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

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

// ------------------------------------------------------------------ int8 arithmetic ----
// The 8-bit window decoders (turbodecoder_win.h WINIMP sse8: 16 sub-blocks, avx8: 32), driven
// by srslte_tdec_iteration_8bit (turbodecoder.c:439-464, turbodecoder_iter.h with LLR_IS_8BIT),
// run as k_win_bidir<..., B8 = true>. Reference semantics: "-INF" = 0, so every start state
// (known or estimated) is all-zero; normalisation subtracts the maximum state after every step
// k != 0; output (m1 - m0) >> 1 per byte; the tail trellis adds with MAKE_FUNC(sadd)
// (:196-203: clamps upwards, wraps downwards). The half-iteration subtractions
// (srslte_vec_sub_bbb) saturate below K & ~31 and wrap above (AVX2 vector body + scalar tail,
// vector_simd.c:165-191); the index that decides is the reference's array index: j for DEC1's
// ext1 - app1, fwd[j] for DEC2's.
// Representation: an int8 value v is held as v << 8 in a packed int16 lane (two CBs per lane as
// everywhere). Then the int16 saturating add clamps exactly at the int8 limits: the sum is exact
// in range, clamps to -128 << 8 below, and to 0x7FFF above, which one AND with 0xFF00 turns into
// 127 << 8 — two packed ops per saturating int8 add, max is one, wrap-around subtraction is the
// plain int16 one, and a subtraction whose result cannot be positive (normalisation) needs no
// mask. SP0 / P1 / T come from the shared loaders unscaled (shifted on load); A and X2, private
// to the int8 decoders between half-iterations, stay scaled.
__device__ __forceinline__ s2 bmask(s2 v) {
  return __builtin_bit_cast(s2, __builtin_bit_cast(uint32_t, v) & 0xFF00FF00u);
}
__device__ __forceinline__ s2 badd(s2 a, s2 b) { return bmask(sadd(a, b)); }
__device__ __forceinline__ s2 bsub(s2 a, s2 b) { return bmask(ssub(a, b)); }
__device__ __forceinline__ s2 bscale(s2 v) { return v << 8; }
__device__ __forceinline__ short tail8(short a, short b) { // unscaled operands
  const int z = a + b;
  return z > 127 ? (short)127 : (short)(signed char)(unsigned char)(z & 255);
}
__device__ __forceinline__ s2 tadd8(s2 a, s2 b) { return s2{tail8(a.x, b.x), tail8(a.y, b.y)}; }
__device__ __forceinline__ void b_norm(int k, St8 &o) {
  if (k != 0) {
    s2 m = smax(smax(smax(o.s[0], o.s[1]), smax(o.s[2], o.s[3])),
                smax(smax(o.s[4], o.s[5]), smax(o.s[6], o.s[7])));
#pragma unroll
    for (int i = 0; i < 8; i++) o.s[i] = ssub(o.s[i], m); // <= 0: only the lower clamp can act
  }
}
// max(badd(a, b), badd(c, d)) == bmask(max(sadd(a, b), sadd(c, d))) for masked operands (bmask
// is monotone and equals badd on each sum), so each new state is masked once
__device__ __forceinline__ void b_beta_step(St8 &o, s2 x, s2 y) {
  s2 xy = badd(x, y);
  s2 b0 = o.s[0], b1 = o.s[1], b2 = o.s[2], b3 = o.s[3];
  s2 b4 = o.s[4], b5 = o.s[5], b6 = o.s[6], b7 = o.s[7];
  o.s[0] = bmask(smax(sadd(b4, xy), b0));
  o.s[1] = bmask(smax(b4, sadd(b0, xy)));
  o.s[2] = bmask(smax(sadd(b5, y), sadd(b1, x)));
  o.s[3] = bmask(smax(sadd(b5, x), sadd(b1, y)));
  o.s[4] = bmask(smax(sadd(b6, x), sadd(b2, y)));
  o.s[5] = bmask(smax(sadd(b6, y), sadd(b2, x)));
  o.s[6] = bmask(smax(b7, sadd(b3, xy)));
  o.s[7] = bmask(smax(sadd(b7, xy), b3));
}
// branch sums left unmasked: each is exact or saturated at 0x7FFF / -32768, and is only combined
// with masked values (stored betas) before a max and one final mask (see b_beta_step), so every
// result equals the all-masked computation
__device__ __forceinline__ void b_alpha_branches(const St8 &o, s2 x, s2 y, s2 mb[8], s2 nw[8]) {
  s2 xy = badd(x, y);
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
// turbodecoder_win.h:263-307 with int8 sadd (unscaled tail values), states returned scaled
__device__ __forceinline__ void b_tail_trellis(const s2 *tail, int xoff, St8 &o) {
  st_fill(o, 0, 0);
#pragma unroll
  for (int j = 2; j >= 0; j--) {
    s2 x = tail[xoff + 2 * j], y = tail[xoff + 2 * j + 1], xy = tadd8(x, y);
    s2 b0 = o.s[0], b1 = o.s[1], b2 = o.s[2], b3 = o.s[3];
    s2 b4 = o.s[4], b5 = o.s[5], b6 = o.s[6], b7 = o.s[7];
    o.s[0] = smax(tadd8(b4, xy), b0);
    o.s[1] = smax(b4, tadd8(b0, xy));
    o.s[2] = smax(tadd8(b5, y), tadd8(b1, x));
    o.s[3] = smax(tadd8(b5, x), tadd8(b1, y));
    o.s[4] = smax(tadd8(b6, x), tadd8(b2, y));
    o.s[5] = smax(tadd8(b6, y), tadd8(b2, x));
    o.s[6] = smax(b7, tadd8(b3, xy));
    o.s[7] = smax(tadd8(b7, xy), b3);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) o.s[i] = o.s[i] << 8;
}
// normalisation by the maximum state (int8 windows, every step k != 0)
__device__ __forceinline__ void b_norm_max(St8 &o) {
  s2 m = smax(smax(smax(o.s[0], o.s[1]), smax(o.s[2], o.s[3])),
              smax(smax(o.s[4], o.s[5]), smax(o.s[6], o.s[7])));
#pragma unroll
  for (int i = 0; i < 8; i++) o.s[i] = ssub(o.s[i], m);
}

// ------------------------------------------------------------------ input policy ----
// Per-step inputs of one constituent decoder run. DEC1: x = syst (+) A, y = par0, operand of
// the output stage = A, scatter table = rev. DEC2: x = app2, y = par1, operand = app2, table =
// fwd. WRAP selects the SSE/generic wrapping add for x (tdec_sse_gamma :321-325, gen.c:72-74)
// instead of the windowed decoders' saturating one (win.h:390-393).
struct StepIn {
  s2 x, y, e;
};

// MODE: 0 = DEC1, 1 = DEC2, 2 = DEC1 of the first half-iteration (app1 is still all zero, so
// A is neither read nor needed: turbodecoder_iter.h:318-323 passes NULL as app).
template <int MODE, bool WRAP>
__device__ __forceinline__ StepIn load_step(const s4 *__restrict__ sp0, const s2 *__restrict__ x2,
                                            const s2 *__restrict__ p1, const s2 *__restrict__ A,
                                            int i) {
  StepIn r;
  if (MODE == 1) {
    r.x = x2[i];
    r.y = p1[i];
    r.e = r.x;
  } else {
    s4 v = sp0[i];
    s2 a = MODE == 2 ? splat(0) : A[i];
    r.x = WRAP ? wadd(lo2(v), a) : sadd(a, lo2(v));
    r.y = hi2(v);
    r.e = a;
  }
  return r;
}

// the same inputs for the int8 windows (B8): values scaled by 256, the a priori added with int8
// saturation; X2 already holds scaled values
template <int MODE, bool B8>
__device__ __forceinline__ StepIn load_w(const s4 *__restrict__ sp0, const s2 *__restrict__ x2,
                                         const s2 *__restrict__ p1, const s2 *__restrict__ A, int i) {
  if (!B8) return load_step<MODE, false>(sp0, x2, p1, A, i);
  StepIn r;
  if (MODE == 1) {
    r.x = x2[i];
    r.y = bscale(p1[i]);
    r.e = r.x;
  } else {
    s4 v = sp0[i];
    s2 a = MODE == 2 ? splat(0) : A[i];
    r.x = MODE == 2 ? bscale(lo2(v)) : badd(a, bscale(lo2(v)));
    r.y = bscale(hi2(v));
    r.e = a;
  }
  return r;
}

// Output stage (turbodecoder_iter.h:315-341): DEC1 ext1 -> app2 (interleave, minus app1);
// DEC2 ext2 -> A (deinterleave, minus the a priori it was fed).
template <bool DEC2>
__device__ __forceinline__ void store_out(s2 *__restrict__ x2, s2 *__restrict__ A, int t, s2 llr,
                                          s2 e) {
  s2 v = wsub(llr, e);
  if (DEC2)
    A[t] = v;
  else
    x2[t] = v;
}

// Decision plane D: the hard decisions of the half-iteration, packed in the decoder's own
// order (chain d, step k): word [pair][d][k / 16] holds CB x's decisions of steps 16h..16h+15 in
// bits 0-15 and CB y's in bits 16-31. llr > 0 is the reference's decision on ext1 / app1
// (turbodecoder.c:353-360), since A + app2 reproduces llr exactly modulo 2^16. k_decide maps
// natural positions onto it (directly after DEC1, through dmap after DEC2).
// dec_bits: 1 at bit 0 (x) / bit 16 (y) where llr > 0. Two packed ops, written as asm: left to
// itself the compiler turns the clamp into per-half compares, selects and a permute (6 ops).
__device__ __forceinline__ uint32_t dec_bits(s2 llr) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0\n\tv_pk_min_i16 %0, %0, 1 op_sel_hi:[1,0]"
      : "=v"(r)
      : "v"(__builtin_bit_cast(uint32_t, llr)));
  return r;
}
__device__ __forceinline__ int dec_words(int K, int NB) { return NB * ((K / NB + 15) / 16); }

// ------------------------------------------------------------------ windowed, bidirectional ----
// Windowed decoder (turbodecoder_win.h), two waves per 64 sub-block chains: wave 0 runs the forward
// (alpha) recursion, wave 1 the backward (beta) recursion, both starting at their end of the
// sub-block and meeting at M (a multiple of CW near L/2). In its first half each wave only
// recurses and checkpoints its metric every CW steps into LDS (alpha: entering state; beta: the
// value the reference stores, before normalisation); after a workgroup barrier each wave emits
// the LLRs of the other wave's first half, recomputing the other metric CW steps at a time from
// those checkpoints. Every position is visited once per direction with the reference's
// normalisation schedule, so all metrics are the reference's; the serial chain is half as long
// and the checkpoints never touch HBM.
template <int CW>
struct ChunkW {
  s2 x[CW], y[CW], e[CW];
  int t[CW];
};

#ifdef TD_TIMING
// debug build only (make timing): shader-clock stamps per wave of the bidirectional decoder
__device__ unsigned long long td_times[2048 * 8];
#define TD_T(k)                                                                                    \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) {                                           \
      td_times[(blockIdx.x * 2 + role) * 8 + (k)] = clock64();                                     \
      if ((k) == 0 || (k) == 4) td_times[(blockIdx.x * 2 + role) * 8 + 5 + (k) / 4] = wall_clock64(); \
    }                                                                                              \
  } while (0)
#else
#define TD_T(k)
#endif

// The body of k_win_bidir: every pointer a __restrict__ parameter, so the scoped no-alias
// facts survive inlining (the group tables would otherwise hide them from the scheduler).
template <int NB, int DIV, int MODE, int CW, bool DOUT, bool B8>
__device__ __forceinline__ void win_bidir_body(const s4 *__restrict__ sp0, s2 *__restrict__ xp1,
                                               const s2 *__restrict__ p1, s2 *__restrict__ A,
                                               uint32_t *__restrict__ D, const s2 *__restrict__ tl,
                                               gptr_t<uint16_t> __restrict__ tbl, s4 *__restrict__ cks,
                                               int K, int d, bool wr, int role, int lane) {
  const int L = K / NB;
  const int nc = (L + CW - 1) / CW;
  const int qm = nc / 2; // meeting chunk: M = CW*qm
  const int tail_xoff = MODE == 1 ? 6 : 0;
  const int K32 = K & ~31; // B8: srslte_vec_sub_bbb saturates below, wraps above (AVX2 body)
  // arithmetic of the variant: 16-bit windows (saturating int16, state-0 normalisation every
  // second step) or B8, the int8 windows (int8 saturation on scaled lanes, maximum-state
  // normalisation after every step)
  auto astep = [&](St8 &o, s2 x, s2 y) {
    if (B8) {
      s2 mb[8], nw[8];
      b_alpha_branches(o, x, y, mb, nw);
#pragma unroll
      for (int i = 0; i < 8; i++) o.s[i] = bmask(smax(mb[i], nw[i]));
    } else {
      win_alpha_step(o, x, y);
    }
  };
  auto bstep = [&](St8 &o, s2 x, s2 y) {
    if (B8)
      b_beta_step(o, x, y);
    else
      win_beta_step(o, x, y);
  };
  auto pnorm = [&](int k, St8 &o) { // prepass normalisation at step k
    if (B8)
      b_norm(k, o);
    else
      win_norm(k, o);
  };

  auto ck_put = [&](int slot, const St8 &o) {
    s4 *p = &cks[((slot * 2) * 64 + lane) * 2];
    p[0] = s4{o.s[0].x, o.s[0].y, o.s[1].x, o.s[1].y};
    p[1] = s4{o.s[2].x, o.s[2].y, o.s[3].x, o.s[3].y};
    s4 *q = &cks[((slot * 2 + 1) * 64 + lane) * 2];
    q[0] = s4{o.s[4].x, o.s[4].y, o.s[5].x, o.s[5].y};
    q[1] = s4{o.s[6].x, o.s[6].y, o.s[7].x, o.s[7].y};
  };
  auto ck_get = [&](int slot, St8 &o) {
    const s4 *p = &cks[((slot * 2) * 64 + lane) * 2];
    const s4 *q = &cks[((slot * 2 + 1) * 64 + lane) * 2];
    s4 a = p[0], b = p[1], c = q[0], e = q[1];
    o.s[0] = lo2(a);
    o.s[1] = hi2(a);
    o.s[2] = lo2(b);
    o.s[3] = hi2(b);
    o.s[4] = lo2(c);
    o.s[5] = hi2(c);
    o.s[6] = lo2(e);
    o.s[7] = hi2(e);
  };
  auto load_x8 = [&](ChunkW<8> &c, int col, int k0) { // prepass chunks (0 <= k0, k0 + 7 < L)
    const int i0 = k0 * NB + col;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      StepIn s = load_w<MODE, B8>(sp0 + i0, xp1 + i0, p1 + i0, A + i0, j * NB);
      c.x[j] = s.x;
      c.y[j] = s.y;
    }
  };
  // chunk loads: a full chunk addresses its 16 steps as one base + constant offsets (no
  // per-step index arithmetic); the last, partial chunk and the backward wave's prefetch past
  // the start (chunk -1, never used) clamp k to [0, L - 1]. Not for MODE 0 (DEC1 with A):
  // there the compiler hoists the offset loads and runs out of registers (measured +30%).
  auto load_xy = [&](ChunkW<CW> &c, int q) {
    if (MODE != 0 && q >= 0 && CW * q + CW <= L) { // (the backward wave prefetches chunk -1)
      const int i0 = CW * q * NB + d;
#pragma unroll
      for (int j = 0; j < CW; j++) {
        StepIn s = load_w<MODE, B8>(sp0 + i0, xp1 + i0, p1 + i0, A + i0, j * NB);
        c.x[j] = s.x;
        c.y[j] = s.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < CW; j++) {
        int k = min(max(CW * q + j, 0), L - 1);
        StepIn s = load_w<MODE, B8>(sp0, xp1, p1, A, k * NB + d);
        c.x[j] = s.x;
        c.y[j] = s.y;
      }
    }
  };
  auto load_full = [&](ChunkW<CW> &c, int q) {
    if (MODE != 0 && q >= 0 && CW * q + CW <= L) { // (the backward wave prefetches chunk -1)
      const int i0 = CW * q * NB + d;
#pragma unroll
      for (int j = 0; j < CW; j++) {
        StepIn s = load_w<MODE, B8>(sp0 + i0, xp1 + i0, p1 + i0, A + i0, j * NB);
        c.x[j] = s.x;
        c.y[j] = s.y;
        c.e[j] = s.e;
        c.t[j] = tbl[i0 + j * NB];
      }
    } else {
#pragma unroll
      for (int j = 0; j < CW; j++) {
        int k = min(max(CW * q + j, 0), L - 1);
        int i = k * NB + d;
        StepIn s = load_w<MODE, B8>(sp0, xp1, p1, A, i);
        c.x[j] = s.x;
        c.y[j] = s.y;
        c.e[j] = s.e;
        c.t[j] = tbl[i];
      }
    }
  };
  auto norm_by = [&](St8 &o, s2 z) {
#pragma unroll
    for (int i = 0; i < 8; i++) o.s[i] = ssub(o.s[i], z);
  };
  // normalisation operand at step k = CW*q + j, k even (win.h:244-261: never at k == 0)
  auto norm_op = [&](const St8 &o, int q, int j) -> s2 {
    return (j == 0 && q == 0) ? splat(0) : o.s[0];
  };
  // alpha after step k = CW q + j
  auto nrm_fwd = [&](St8 &o, int q, int j) {
    if (B8) {
      if (!(q == 0 && j == 0)) b_norm_max(o);
    } else if ((j & 1) == 0) {
      norm_by(o, norm_op(o, q, j));
    }
  };
  // after a step k != 0 that is even when `even`
  auto nrm_k = [&](St8 &o, bool even) {
    if (B8)
      b_norm_max(o);
    else if (even)
      norm_by(o, o.s[0]);
  };
  // LLR at position k from alpha_k (al), the chunk's inputs and stored beta[k+1] (be)
  static_assert(CW == 16, "decision words hold 16 steps");
  const int G16 = (L + 15) / 16;
  auto llr_out = [&](const ChunkW<CW> &c, const St8 &al, const St8 &be, int j, uint32_t &dacc,
                     s2 mb[8], s2 nw[8], int idx) {
    if (B8)
      b_alpha_branches(al, c.x[j], c.y[j], mb, nw);
    else
      win_alpha_branches(al, c.x[j], c.y[j], mb, nw);
    // max over the 8 branches as a tree (max is exact, so any order is the reference's)
    s2 t0[8], t1[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      t0[i] = sadd(be.s[i], mb[i]); // B8: masked once after the tree (bmask is monotone)
      t1[i] = sadd(be.s[i], nw[i]);
    }
#pragma unroll
    for (int w = 4; w >= 1; w >>= 1)
#pragma unroll
      for (int i = 0; i < w; i++) {
        t0[i] = smax(t0[i], t0[i + w]);
        t1[i] = smax(t1[i], t1[i + w]);
      }
    s2 v = B8 ? bsub(bmask(t1[0]), bmask(t0[0])) : ssub(t1[0], t0[0]);
    if (B8)
      v = bmask(v >> 1); // per-byte srai 1 (simd_rb_shift)
    else if (DIV)
      v = v >> 1; // win.h:565-567 srai 1 (SSE16 window)
    if (wr) {
      if (B8) { // ext - app with the reference's saturate / wrap split (K32, see above)
        const int t = c.t[j];
        const bool sat = (MODE == 1 ? t : idx) < K32;
        const s2 out = MODE == 2 ? v : (sat ? bsub(v, c.e[j]) : wsub(v, c.e[j]));
        if (MODE == 1)
          A[t] = out;
        else
          xp1[t] = out;
      } else {
        store_out<MODE == 1>(xp1, A, c.t[j], v, c.e[j]);
      }
    }
    if (DOUT) dacc |= dec_bits(v) << j;
  };

  St8 o;
  if (role == 0) {
    // ================= forward wave =================
    {
      // win.h:501-506,512-584 (loop_len = 40) over the last 40 steps of sub-block d-1;
      // move_left (:469-495); sub-block 0 starts in state 0 (:496-500)
      const int dp = d > 0 ? d - 1 : 0;
      st_fill(o, B8 ? 0 : -TD_INF, B8 ? 0 : -TD_INF);
      ChunkW<8> c0, c1;
      load_x8(c0, dp, L - TD_OVERLAP);
#pragma unroll
      for (int q = 0; q < 5; q += 2) {
        if (q < 4) load_x8(c1, dp, L - TD_OVERLAP + 8 * (q + 1));
#pragma unroll
        for (int j = 0; j < 8; j++) {
          astep(o, c0.x[j], c0.y[j]);
          pnorm(8 * q + j, o);
        }
        if (q < 4) {
          if (q < 3) load_x8(c0, dp, L - TD_OVERLAP + 8 * (q + 2));
#pragma unroll
          for (int j = 0; j < 8; j++) {
            astep(o, c1.x[j], c1.y[j]);
            pnorm(8 * (q + 1) + j, o);
          }
        }
      }
      if (d == 0) st_fill(o, 0, B8 ? 0 : -TD_INF);
    }
    TD_T(1);
    // first half: chunks 0 .. qm-1, checkpoint the entering state of each
    {
      auto fwd_chunk = [&](ChunkW<CW> &c, int q) {
        ck_put(q, o);
#pragma unroll
        for (int j = 0; j < CW; j++) {
          astep(o, c.x[j], c.y[j]);
          nrm_fwd(o, q, j);
        }
      };
      ChunkW<CW> c0, c1;
      int q = 0;
      load_xy(c0, 0);
      for (; q + 1 < qm; q += 2) {
        load_xy(c1, q + 1);
        fwd_chunk(c0, q);
        load_xy(c0, q + 2);
        fwd_chunk(c1, q + 1);
      }
      if (q < qm) fwd_chunk(c0, q);
    }
    TD_T(2);
    __syncthreads();
    TD_T(3);
    // second half: segments qm .. nc-1 with betas recomputed from the backward checkpoints
    {
      auto seg = [&](ChunkW<CW> &c, int q, bool last) {
        const int s0 = CW * q;
        const int n = last ? L - s0 : CW;
        St8 bst[CW]; // bst[j] = stored beta[s0+1+j]
        uint32_t dacc = 0;
        St8 run;
        ck_get(min(q + 1, nc), run);
#pragma unroll
        for (int j = CW - 1; j >= 0; j--)
          if (j == n - 1) bst[j] = run;
        if (!last) nrm_k(run, true); // s1 = s0+CW < L: even, non-zero
#pragma unroll
        for (int j = CW - 2; j >= 0; j--) {
          if (j <= n - 2) {
            bstep(run, c.x[j + 1], c.y[j + 1]);
            bst[j] = run;
            nrm_k(run, ((j + 1) & 1) == 0); // k = s0+1+j >= 1
          }
        }
#pragma unroll
        for (int j = 0; j < CW; j++) {
          if (j < n) {
            s2 mb[8], nw[8];
            llr_out(c, o, bst[j], j, dacc, mb, nw, (s0 + j) * NB + d);
#pragma unroll
            for (int i = 0; i < 8; i++) o.s[i] = B8 ? bmask(smax(mb[i], nw[i])) : smax(mb[i], nw[i]);
            nrm_fwd(o, q, j);
          }
        }
        if (DOUT && wr) D[d * G16 + q] = dacc;
      };
      ChunkW<CW> c0, c1;
      int q = qm;
      load_full(c0, q);
      for (; q + 2 < nc; q += 2) {
        load_full(c1, q + 1);
        seg(c0, q, false);
        load_full(c0, q + 2);
        seg(c1, q + 1, false);
      }
      if (q == nc - 2) {
        load_full(c1, q + 1);
        seg(c0, q, false);
        seg(c1, q + 1, true);
      } else {
        seg(c0, q, true);
      }
    }
  } else {
    // ================= backward wave =================
    {
      // win.h:376-384,386-433 (loop_len = 40) over the first 40 steps of sub-block d+1;
      // move_right (:333-366); the last sub-block starts from the tail trellis (:350-355)
      const int dn = d + 1 < NB ? d + 1 : d;
      st_fill(o, B8 ? 0 : -TD_INF, B8 ? 0 : -TD_INF);
      ChunkW<8> c0, c1;
      load_x8(c0, dn, 32);
#pragma unroll
      for (int q = 4; q >= 0; q -= 2) {
        if (q > 0) load_x8(c1, dn, 8 * (q - 1));
#pragma unroll
        for (int j = 7; j >= 0; j--) {
          bstep(o, c0.x[j], c0.y[j]);
          pnorm(8 * q + j, o);
        }
        if (q > 0) {
          if (q > 1) load_x8(c0, dn, 8 * (q - 2));
#pragma unroll
          for (int j = 7; j >= 0; j--) {
            bstep(o, c1.x[j], c1.y[j]);
            pnorm(8 * (q - 1) + j, o);
          }
        }
      }
      St8 t;
      if (B8)
        b_tail_trellis(tl, tail_xoff, t);
      else
        win_tail_trellis(tl, tail_xoff, t);
      if (d == NB - 1) o = t;
    }
    ck_put(nc, o); // beta[L] (win.h:372-374)
    TD_T(1);
    // first half: chunks nc-1 .. qm (steps L-1 .. M); bpre ends as beta[M] before normalisation
    St8 bpre;
    {
      auto bwd_chunk = [&](ChunkW<CW> &c, int q, int n, bool keep) { // q > 0: norm never at 0
#pragma unroll
        for (int j = CW - 1; j >= 0; j--) {
          if (j < n) {
            bstep(o, c.x[j], c.y[j]);
            if (j == 0) {
              if (keep)
                bpre = o;
              else
                ck_put(q, o);
            }
            nrm_k(o, (j & 1) == 0);
          }
        }
      };
      ChunkW<CW> c0, c1;
      const int qt = nc - 1; // top chunk, possibly partial; qt > qm
      load_xy(c0, qt);
      load_xy(c1, qt - 1);
      bwd_chunk(c0, qt, L - CW * qt, false);
      int q = qt - 1; // in c1
      for (; q - 1 > qm; q -= 2) {
        load_xy(c0, q - 1);
        bwd_chunk(c1, q, CW, false);
        load_xy(c1, q - 2);
        bwd_chunk(c0, q - 1, CW, false);
      }
      if (q > qm) {
        load_xy(c0, q - 1);
        bwd_chunk(c1, q, CW, false);
        bwd_chunk(c0, qm, CW, true);
      } else {
        bwd_chunk(c1, qm, CW, true);
      }
    }
    TD_T(2);
    __syncthreads();
    TD_T(3);
    // second half: segments qm-1 .. 0 (full), alphas recomputed from the forward checkpoints
    {
      auto seg = [&](ChunkW<CW> &c, int q) {
        St8 ast[CW]; // ast[j] = alpha entering step CW*q+j
        uint32_t dacc = 0;
        ck_get(q, ast[0]);
#pragma unroll
        for (int j = 0; j < CW - 1; j++) {
          ast[j + 1] = ast[j];
          astep(ast[j + 1], c.x[j], c.y[j]);
          nrm_fwd(ast[j + 1], q, j);
        }
#pragma unroll
        for (int j = CW - 1; j >= 0; j--) {
          s2 mb[8], nw[8];
          llr_out(c, ast[j], bpre, j, dacc, mb, nw, (CW * q + j) * NB + d); // bpre = stored beta[k+1]
          // running beta at k+1 (normalised when k+1 is even; k+1 >= 1), then beta[k]
          St8 run = bpre;
          nrm_k(run, ((j + 1) & 1) == 0);
          bstep(run, c.x[j], c.y[j]);
          bpre = run;
        }
        if (DOUT && wr) D[d * G16 + q] = dacc;
      };
      ChunkW<CW> c0, c1;
      int q = qm - 1;
      load_full(c0, q);
      for (; q - 1 >= 0; q -= 2) {
        load_full(c1, q - 1);
        seg(c0, q);
        load_full(c0, q - 2);
        seg(c1, q - 1);
      }
      if (q == 0) seg(c0, 0);
    }
  }
}

template <int NB, int DIV, int MODE, int CW, bool DOUT, bool B8>
__global__ __launch_bounds__(128) void k_win_bidir(const TdGroup *__restrict__ groups, int ngroups,
                                                   const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                   s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                   const s2 *__restrict__ T, size_t plane,
                                                   const uint8_t *__restrict__ pair_done) {
  // checkpoint slots in (dynamic) LDS, [slot][half][lane] x 16 B (conflict-free b128 accesses);
  // nc + 1 slots of 2 KiB: 50 KiB at K = 6144 with 16 sub-blocks
  extern __shared__ s4 cks[];
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); // 0: alpha, 1: beta
  TD_T(0);
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int K = G.K, npairs = G.npairs;
  const int blk = blockIdx.x - G.blk_half;
  const int lane = threadIdx.x & 63;
  const int gl = blk * 64 + lane;
  const int nlanes = npairs * NB;
  const bool live = gl < nlanes;
  const int g = live ? gl : nlanes - 1; // dead lanes compute on valid data, store nothing
  const int pair = g / NB;              // within the group
  const int d = g % NB;
  const uint8_t *pdone = pair_done ? pair_done + G.pair0 : nullptr;
  {
    // whole block finished (early stop): both waves leave before the barrier
    const int p0 = (blk * 64) / NB;
    const int p1 = min((blk * 64 + 63) / NB, npairs - 1);
    bool all_done = pdone != nullptr;
    if (pdone)
      for (int p = p0; p <= p1; p++) all_done = all_done && pdone[p];
    if (all_done) return;
  }
  const bool wr = live && !(pdone && pdone[pair]);
  const size_t base = (size_t)G.elem0 + (size_t)pair * K;
  const s4 *sp0 = SP0 + base;
  s2 *xp1 = XP1 + base;                  // app2 (DEC1 output)
  const s2 *p1 = XP1 + plane + base;     // par1
  s2 *A = Aarr + base;
  uint32_t *D = DOUT ? Darr + G.dw0 + (size_t)pair * dec_words(K, NB) : nullptr;
  const s2 *tl = T + (size_t)(G.pair0 + pair) * 12;
  const gptr_t<uint16_t> tbl = gptr(MODE == 1 ? G.fwd : G.rev);
  win_bidir_body<NB, DIV, MODE, CW, DOUT, B8>(sp0, xp1, p1, A, D, tl, tbl, cks, K, d, wr, role, lane);
  TD_T(4);
}

// ------------------------------------------------------------------ SSE non-window ----
// turbodecoder_sse.c:97-407, one lane per CB pair, natural index (NB = 1). Branch metrics from
// x (wrapping app add, tdec_sse_gamma :321-325) and y; tail gammas use C division (:349-352).
// scratch: alpha (K+1)*8 short2 per pair, lane-interleaved.
template <int MODE>
__global__ __launch_bounds__(64) void k_sse_halfit(const TdGroup *__restrict__ groups, int ngroups,
                                                   const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                   s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                   const s2 *__restrict__ T, size_t plane,
                                                   s2 *__restrict__ scratch_base,
                                                   const uint8_t *__restrict__ pair_done) {
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int K = G.K, npairs = G.npairs;
  const int pair = (blockIdx.x - G.blk_half) * blockDim.x + threadIdx.x; // within the group
  if (pair >= npairs) return;
  if (pair_done && pair_done[G.pair0 + pair]) return;
  const size_t base = (size_t)G.elem0 + (size_t)pair * K;
  const s4 *sp0 = SP0 + base;
  s2 *xp1 = XP1 + base;                  // app2 (DEC1 output)
  const s2 *p1 = XP1 + plane + base;     // par1
  s2 *A = Aarr + base;
  uint32_t *D = Darr ? Darr + G.dw0 + (size_t)pair * dec_words(K, 1) : nullptr;
  const s2 *tl = T + (size_t)(G.pair0 + pair) * 12;
  const gptr_t<uint16_t> tbl = gptr(MODE == 1 ? G.fwd : G.rev);
  s2 *scratch = scratch_base + G.sc0;
  const int tail_xoff = MODE == 1 ? 6 : 0;
  auto AL = [&](int k, int i) -> s2 & { return scratch[((size_t)k * 8 + i) * npairs + pair]; };
  s2 a[8];
  a[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) a[i] = splat(-TD_INF);
#pragma unroll
  for (int i = 0; i < 8; i++) AL(0, i) = a[i];
  for (int k = 0; k < K; k++) { // :211-297
    StepIn s = load_step<MODE, true>(sp0, xp1, p1, A, k);
    s2 g1 = wadd(s.x, s.y) >> 1, g0 = wsub(s.x, s.y) >> 1;
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
  uint32_t dacc = 0;
  for (int k = K + 2; k >= 0; k--) { // :105-206
    s2 g0, g1, e = splat(0);
    if (k >= K) {
      s2 x = tl[tail_xoff + 2 * (k - K)], y = tl[tail_xoff + 2 * (k - K) + 1];
      g0 = s2{(short)(((int)x.x - y.x) / 2), (short)(((int)x.y - y.y) / 2)};
      g1 = s2{(short)(((int)x.x + y.x) / 2), (short)(((int)x.y + y.y) / 2)};
    } else {
      StepIn s = load_step<MODE, true>(sp0, xp1, p1, A, k);
      g1 = wadd(s.x, s.y) >> 1;
      g0 = wsub(s.x, s.y) >> 1;
      e = s.e;
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
      // hMax(bn) - hMax(bp) with hMax(v) = 0x7FFF - max(v) (minpos_epu16 trick, :97-102)
      s2 llr = wsub(wsub(splat(0x7FFF), mn), wsub(splat(0x7FFF), mp));
      store_out<MODE == 1>(xp1, A, tbl[k], llr, e);
      if (D) { // k descends: flush each 16-step group at its first step
        dacc |= dec_bits(llr) << (k & 15);
        if ((k & 15) == 0) {
          D[k >> 4] = dacc;
          dacc = 0;
        }
      }
      if ((k & 3) == 0) {
        s2 z = b[0];
#pragma unroll
        for (int i = 0; i < 8; i++) b[i] = wsub(b[i], z);
      }
    }
  }
}

// ------------------------------------------------------------------ generic ----
// turbodecoder_gen.c:59-236, one lane per CB pair, natural index, wrapping int16; app is added
// for k < K only (:72-74), which is exactly the range the input policy covers.
// scratch: beta (K+4)*8 short2 per pair.
template <int MODE>
__global__ __launch_bounds__(64) void k_gen_halfit(const TdGroup *__restrict__ groups, int ngroups,
                                                   const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                   s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                   const s2 *__restrict__ T, size_t plane,
                                                   s2 *__restrict__ scratch_base,
                                                   const uint8_t *__restrict__ pair_done) {
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int K = G.K, npairs = G.npairs;
  const int pair = (blockIdx.x - G.blk_half) * blockDim.x + threadIdx.x; // within the group
  if (pair >= npairs) return;
  if (pair_done && pair_done[G.pair0 + pair]) return;
  const size_t base = (size_t)G.elem0 + (size_t)pair * K;
  const s4 *sp0 = SP0 + base;
  s2 *xp1 = XP1 + base;                  // app2 (DEC1 output)
  const s2 *p1 = XP1 + plane + base;     // par1
  s2 *A = Aarr + base;
  uint32_t *D = Darr ? Darr + G.dw0 + (size_t)pair * dec_words(K, 1) : nullptr;
  const s2 *tl = T + (size_t)(G.pair0 + pair) * 12;
  const gptr_t<uint16_t> tbl = gptr(MODE == 1 ? G.fwd : G.rev);
  s2 *scratch = scratch_base + G.sc0;
  const int tail_xoff = MODE == 1 ? 6 : 0;
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
      StepIn s = load_step<MODE, true>(sp0, xp1, p1, A, k);
      x = s.x;
      y = s.y;
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
  uint32_t dacc = 0;
  for (int k = 1; k < K + 1; k++) {
    StepIn s = load_step<MODE, true>(sp0, xp1, p1, A, k - 1);
    s2 x = s.x, y = s.y, xy_ = wadd(x, y);
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
    store_out<MODE == 1>(xp1, A, tbl[k - 1], wsub(m1, m0), s.e);
    if (D) {
      dacc |= dec_bits(wsub(m1, m0)) << ((k - 1) & 15);
      if (((k - 1) & 15) == 15 || k == K) {
        D[(k - 1) >> 4] = dacc;
        dacc = 0;
      }
    }
  }
}

// ------------------------------------------------------------------ load ----
// User layout -> SP0 / P1 / T. Natural input ([s,p0,p1]*K + 12 tail;
// turbodecoder_gen.c:240-259, win.h:634-674) is transposed through LDS: a workgroup takes 64
// consecutive steps k of all NB sub-blocks of one pair, reads NB runs of 64 natural positions
// (coalesced), and writes the 64*NB SB-ordered elements contiguously. SB input (rm_turbo's
// layout, streams at s*(K+32), tails at 3*(K+32); turbodecoder_iter.h:271-280) is a straight copy.
#define LOAD_KT 64
// input row of code block c: strided rows, or a per-CB pointer table (DL-SCH softbuffer rows)
__device__ __forceinline__ gptr_t<int16_t> cb_row(const int16_t *in, size_t stride,
                                                  const int16_t *const *rows, int c) {
  return gptr(rows ? rows[c] : in + (size_t)c * stride);
}
// NB and the tile are compile-time so the run/offset arithmetic is shifts and multiplies; VEC
// reads the natural runs as 8-byte words (rows 8-byte aligned, L a multiple of 4).
template <int NB, bool VEC>
__global__ __launch_bounds__(256) void k_load_nat(const TdGroup *__restrict__ groups, int ngroups,
                                                  const int16_t *__restrict__ in, size_t in_stride,
                                                  const int16_t *const *__restrict__ rows,
                                                  TdArrays arr) {
  // phase 1 copies each (CB, sub-block) run of 3 * LOAD_KT int16 into LDS as it lies (natural
  // order, 8-byte accesses when VEC), rows padded to RS shorts (98 dwords: the phase-2 reads of
  // 16 sub-blocks fall in distinct banks); phase 2 reads the triplets back in sub-block order
  // and writes SP0 / P1 coalesced
  constexpr int RUN = 3 * LOAD_KT; // int16 per (CB, sub-block) run of one tile
  constexpr int RS = RUN + 4;
  __shared__ __attribute__((aligned(16))) short lds[2][NB][RS];
  const TdGroup &G = groups[grp_find<GF_LOAD>(groups, ngroups, blockIdx.x)];
  const int K = G.K, ncb = G.ncb, npairs = G.npairs;
  const int L = K / NB;
  const int ktiles = (L + LOAD_KT - 1) / LOAD_KT;
  const int blk = blockIdx.x - G.blk_load;
  const int pair = blk / ktiles;
  const int kt = blk - pair * ktiles;
  if (pair >= npairs) return;
  const int c0 = G.cb0 + 2 * pair, c1 = 2 * pair + 1 < ncb ? c0 + 1 : c0;
  const int k0 = kt * LOAD_KT;
  const int kn = min(LOAD_KT, L - k0);
  const int n3 = 3 * kn;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const gptr_t<int16_t> src = cb_row(in, in_stride, rows, h ? c1 : c0) + 3 * k0;
    if (VEC) { // src, 3L and 3 k0 all multiples of 4 int16 (the launcher checks)
      typedef uint32_t u2v __attribute__((ext_vector_type(2)));
      constexpr int Q = RUN / 4; // 8-byte words per run
      for (int w = threadIdx.x; w < NB * Q; w += 256) {
        const int dd = w / Q, q = w - dd * Q;
        if (4 * q < n3)
          *(u2v *)&lds[h][dd][4 * q] = *(const __attribute__((address_space(1))) u2v *)(src + dd * 3 * L + 4 * q);
      }
    } else {
      for (int e = threadIdx.x; e < NB * RUN; e += 256) {
        const int dd = e / RUN, r = e - dd * RUN;
        if (r < n3) lds[h][dd][r] = src[dd * 3 * L + r];
      }
    }
  }
  __syncthreads();
  const gmut_t<s4> SP0 = gmut<s4>(arr.SP0);
  const gmut_t<s2> P1 = gmut<s2>(arr.XP1) + arr.plane;
  const size_t base = (size_t)G.elem0 + (size_t)pair * K + (size_t)k0 * NB;
  for (int e = threadIdx.x; e < kn * NB; e += 256) {
    const int kk = e / NB, dd = e - kk * NB;
    const short *a = &lds[0][dd][3 * kk], *b = &lds[1][dd][3 * kk];
    SP0[base + e] = s4{a[0], b[0], a[1], b[1]};
    P1[base + e] = s2{a[2], b[2]};
  }
  if (kt == 0 && threadIdx.x < 12) {
    const int t = threadIdx.x;
    gmut<s2>(arr.T)[(size_t)(G.pair0 + pair) * 12 + t] = s2{cb_row(in, in_stride, rows, c0)[3 * K + t],
                                                         cb_row(in, in_stride, rows, c1)[3 * K + t]};
  }
}

// SB input (rm_turbo's layout, streams at s*(K+32), tails at 3*(K+32); turbodecoder_iter.h:271-280):
// already in SB index order, a straight pair-interleaving copy, two elements per thread.
__global__ __launch_bounds__(256) void k_load_sb(const TdGroup *__restrict__ groups, int ngroups,
                                                 const int16_t *__restrict__ in, size_t in_stride,
                                                 const int16_t *const *__restrict__ rows,
                                                 TdArrays arr) {
  const TdGroup &G = groups[grp_find<GF_LOAD>(groups, ngroups, blockIdx.x)];
  const int K = G.K, ncb = G.ncb, npairs = G.npairs;
  const int per = K / 2;
  const size_t gid = (size_t)(blockIdx.x - G.blk_load) * 256 + threadIdx.x;
  const int pair = (int)(gid / per);
  if (pair >= npairs) return;
  const int i = 2 * (int)(gid - (size_t)pair * per);
  const int c0 = G.cb0 + 2 * pair, c1 = 2 * pair + 1 < ncb ? c0 + 1 : c0;
  const gptr_t<int16_t> a = cb_row(in, in_stride, rows, c0), b = cb_row(in, in_stride, rows, c1);
  const gmut_t<s4> SP0 = gmut<s4>(arr.SP0);
  const gmut_t<s2> P1 = gmut<s2>(arr.XP1) + arr.plane;
  const gmut_t<s2> T = gmut<s2>(arr.T);
  const size_t o = (size_t)G.elem0 + (size_t)pair * K + i;
#pragma unroll
  for (int u = 0; u < 2; u++) {
    SP0[o + u] = s4{a[i + u], b[i + u], a[K + 32 + i + u], b[K + 32 + i + u]};
    P1[o + u] = s2{a[2 * (K + 32) + i + u], b[2 * (K + 32) + i + u]};
  }
  if (i < 12) {
    const int tb = 3 * (K + 32);
    const size_t t = (size_t)(G.pair0 + pair) * 12 + i;
    T[t] = s2{a[tb + i], b[tb + i]};
    T[t + 1] = s2{a[tb + i + 1], b[tb + i + 1]};
  }
}

// The same copy, eight elements of a pair per thread with 16-byte accesses (rows 16-byte aligned,
// as the DL-SCH softbuffer rows are; K is a multiple of 8 for every LTE code block size): six
// 16-byte loads, four 16-byte SP0 stores and two 16-byte P1 stores per thread.
__global__ __launch_bounds__(256) void k_load_sb8(const TdGroup *__restrict__ groups, int ngroups,
                                                  const int16_t *__restrict__ in, size_t in_stride,
                                                  const int16_t *const *__restrict__ rows,
                                                  TdArrays arr) {
  const TdGroup &G = groups[grp_find<GF_LOAD>(groups, ngroups, blockIdx.x)];
  const int K = G.K, ncb = G.ncb, npairs = G.npairs;
  const int per = K / 8;
  const size_t gid = (size_t)(blockIdx.x - G.blk_load) * 256 + threadIdx.x;
  const int pair = (int)(gid / per);
  if (pair >= npairs) return;
  const int i = 8 * (int)(gid - (size_t)pair * per);
  const int c0 = G.cb0 + 2 * pair, c1 = 2 * pair + 1 < ncb ? c0 + 1 : c0;
  const gptr_t<int16_t> a = cb_row(in, in_stride, rows, c0), b = cb_row(in, in_stride, rows, c1);
  typedef short s8v __attribute__((ext_vector_type(8)));
  auto ld8 = [](gptr_t<int16_t> p) { return *(const __attribute__((address_space(1))) s8v *)p; };
  const s8v sa = ld8(a + i), sb = ld8(b + i);
  const s8v pa = ld8(a + K + 32 + i), pb = ld8(b + K + 32 + i);
  const s8v qa = ld8(a + 2 * (K + 32) + i), qb = ld8(b + 2 * (K + 32) + i);
  const size_t o = (size_t)G.elem0 + (size_t)pair * K + i; // multiple of 8: 16-byte aligned
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  const gmut_t<u4v> SP0 = gmut<u4v>((s4 *)arr.SP0 + o);
  const gmut_t<u4v> P1 = gmut<u4v>((s2 *)arr.XP1 + arr.plane + o);
  auto pk = [](short lo, short hi) { return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16); };
#pragma unroll
  for (int u = 0; u < 4; u++) // two short4 (syst.a, syst.b, par0.a, par0.b) per 16-byte store
    SP0[u] = u4v{pk(sa[2 * u], sb[2 * u]), pk(pa[2 * u], pb[2 * u]),
                 pk(sa[2 * u + 1], sb[2 * u + 1]), pk(pa[2 * u + 1], pb[2 * u + 1])};
#pragma unroll
  for (int u = 0; u < 2; u++) // four short2 (par1.a, par1.b) per 16-byte store
    P1[u] = u4v{pk(qa[4 * u], qb[4 * u]), pk(qa[4 * u + 1], qb[4 * u + 1]),
                pk(qa[4 * u + 2], qb[4 * u + 2]), pk(qa[4 * u + 3], qb[4 * u + 3])};
  if (i == 0) { // one thread per pair: the tails
    const int tb = 3 * (K + 32);
    const gmut_t<s2> T = gmut<s2>(arr.T);
#pragma unroll
    for (int t = 0; t < 12; t++) T[(size_t)(G.pair0 + pair) * 12 + t] = s2{a[tb + t], b[tb + t]};
  }
}

// ------------------------------------------------------------------ decide (+ CRC) ----
// Hard decision after half-iteration n (turbodecoder.c:353-360 + decision_byte), MSB first,
// from the decoders' packed decision words D (see dec_bits). One workgroup per CB pair:
//   1. the pair's words (K/16 of them, 1.5 KB at K = 6144) are staged in LDS;
//   2. each wave takes 64 consecutive natural positions p. After DEC1 (even n) position
//      p = d L + k is step k of chain d; after DEC2 dmap[p] gives the chain-major index of the
//      interleaved position that carries it. Two ballots give the 64 decision bits of each CB,
//      lanes 0-15 write the 8+8 output bytes, and the CRC (crc.c:144-155, MSB-first, zero
//      init) is folded from coalesced reads of crc_pw (see below) and reduced.
// With early stop the same workgroup updates the done flags (sch.c:361-391).
__global__ __launch_bounds__(256) void k_decide(int n, const TdGroup *__restrict__ groups,
                                                int ngroups, const uint32_t *__restrict__ Darr,
                                                uint8_t *__restrict__ outb, size_t out_stride,
                                                int early, uint8_t *__restrict__ cb_done,
                                                uint8_t *__restrict__ cb_ok, uint32_t *__restrict__ noi,
                                                int max_halfits, uint8_t *__restrict__ pair_done) {
  __shared__ uint32_t dw[6144 / 16 + 16];
  __shared__ uint32_t red[2][4];
  __shared__ int fin[4]; // [0..1] CB done, [2..3] CB finished at this half-iteration
  const TdGroup &G = groups[grp_find<GF_PAIR>(groups, ngroups, blockIdx.x)];
  const int K = G.K, NB = G.nb, ncb = G.ncb;
  const int pair = blockIdx.x - G.pair0;
  if (pair >= G.npairs) return;
  const int cbs[2] = {G.cb0 + 2 * pair, 2 * pair + 1 < ncb ? G.cb0 + 2 * pair + 1 : -1};
  const bool skip0 = early && cb_done[cbs[0]];
  const bool skip1 = cbs[1] < 0 || (early && cb_done[cbs[1]]);
  if (skip0 && skip1) return;
  const gptr_t<uint16_t> dmap = gptr(G.dmap);
  const int crc_bytes = early ? G.crc_bytes : 0;
  const int L = K / NB, G16 = (L + 15) / 16, nw = NB * G16;
  const uint32_t *src = Darr + G.dw0 + (size_t)pair * nw;
  for (int q = threadIdx.x; q < nw; q += blockDim.x) dw[q] = src[q];
  __syncthreads();
  const bool dec2 = n & 1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int UMAX = (6144 + 256) / 256; // chain-major bits per thread (nw * 16 <= 6400)
  bool out[2] = {!skip0, !skip1};          // natural-order bytes wanted for CB h
  if (crc_bytes) {
    // CRC straight from the decision words (crc.c:144-155 is linear): the XOR of the chain-major
    // weights wc[c] over the set bits c (TdGroup::wc); all loads issued up front
    const gptr_t<uint32_t> wc = gptr(G.wc[dec2 ? 1 : 0]);
    uint32_t c0 = 0, c1 = 0, v[UMAX];
#pragma unroll
    for (int u = 0; u < UMAX; u++) {
      const int c = u * 256 + threadIdx.x;
      v[u] = c < nw * 16 ? wc[c] : 0u;
    }
#pragma unroll
    for (int u = 0; u < UMAX; u++) {
      const int c = u * 256 + threadIdx.x;
      if (c < nw * 16) {
        const uint32_t w = dw[c >> 4] >> (c & 15);
        if (w & 1u) c0 ^= v[u];
        if (w & 0x10000u) c1 ^= v[u];
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      c0 ^= __shfl_xor(c0, o);
      c1 ^= __shfl_xor(c1, o);
    }
    if (lane == 0) {
      red[0][wv] = c0;
      red[1][wv] = c1;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
      const int h = threadIdx.x;
      int done = 1, now = 0;
      if (!(h ? skip1 : skip0)) {
        uint32_t crc = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) crc ^= red[h][w];
        const int cb = cbs[h];
        noi[cb] = (uint32_t)(n + 1);
        if (crc == 0) {
          cb_ok[cb] = 1;
          cb_done[cb] = 1;
          now = 1;
        } else if (n + 1 >= max_halfits) {
          cb_done[cb] = 1;
          now = 1;
        } else {
          done = 0;
        }
      }
      fin[h] = done;
      fin[2 + h] = now;
    }
    __syncthreads();
    if (threadIdx.x == 0 && pair_done) pair_done[blockIdx.x] = (uint8_t)(fin[0] && fin[1]);
    // the bytes of a block matter once, at the half-iteration that ends it (sch.c:361-391: the
    // data of the last iteration run stays)
    out[0] = fin[2] != 0;
    out[1] = fin[3] != 0;
    if (!out[0] && !out[1]) return;
  }
  // Hard decisions in natural order (turbodecoder.c:353-360 + decision_byte), MSB first.
  // DEC1: p = d L + k -> d * 16 G16 + k; d from a float reciprocal (exact: p < 6144, so the
  // fraction of (p + 0.5) / L stays >= 1 / (2 L) away from an integer)
  const float invL = 1.0f / (float)L;
  const int gap = 16 * G16 - L;
  auto chain_index = [&](int p) -> int {
    if (dec2) return (int)dmap[p];
    const int d = (int)(((float)p + 0.5f) * invL);
    return p + d * gap;
  };
  // Position of group u in wave wv: p = wv * 64 + u * 256 + lane (64 consecutive per ballot);
  // every map load of the thread issued before the first use
  constexpr int PMAX = 6144 / 256;
  int ci[PMAX];
#pragma unroll
  for (int u = 0; u < PMAX; u++) {
    const int p = wv * 64 + u * 256 + lane;
    ci[u] = p < K ? chain_index(p) : 0;
  }
#pragma unroll
  for (int u = 0; u < PMAX; u++) {
    const int p0 = wv * 64 + u * 256;
    if (p0 >= K) break;
    const int p = p0 + lane;
    uint32_t dd = 0u;
    if (p < K) {
      const uint32_t w = dw[ci[u] >> 4] >> (ci[u] & 15);
      dd = (w & 1u) | ((w >> 15) & 2u);
    }
    const uint64_t m0 = __ballot(dd & 1u), m1 = __ballot(dd & 2u);
    const int h = lane >> 3, b = lane & 7;
    if (lane < 16 && p0 + 8 * b < K && out[h]) {
      const uint32_t v = (uint32_t)(((h ? m1 : m0) >> (8 * b)) & 0xffu);
      outb[(size_t)cbs[h] * out_stride + (p0 >> 3) + b] = (uint8_t)(__builtin_bitreverse32(v) >> 24);
    }
  }
}

// pair_done = both code blocks finished (seeding after init_done)
__global__ void k_pair_done(const TdGroup *__restrict__ groups, int ngroups, int npairs_total,
                            const uint8_t *__restrict__ cb_done, uint8_t *__restrict__ pair_done) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs_total) return;
  const TdGroup &G = groups[grp_find<GF_PAIR>(groups, ngroups, p)];
  const int lp = p - G.pair0;
  const int c0 = G.cb0 + 2 * lp, c1 = 2 * lp + 1 < G.ncb ? c0 + 1 : c0;
  pair_done[p] = cb_done[c0] && cb_done[c1];
}

// ------------------------------------------------------------------ launchers ----

static inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// dynamic LDS above 64 KiB (the 8-sub-block decoder at large K) needs the per-kernel opt-in
static void allow_big_lds(const void *f) {
  (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

int load_blocks(int K, int nb, int npairs, int sb_input, bool vec16) {
  if (sb_input) return (int)nblk((size_t)npairs * (K / (vec16 ? 8 : 2)), 256);
  return npairs * ((K / nb + LOAD_KT - 1) / LOAD_KT);
}

int halfit_blocks(int nb, int npairs) { return nb > 1 ? (int)nblk((size_t)npairs * nb, 64) : (int)nblk(npairs, 64); }

size_t seq_scratch_elems(int K, int npairs) { return (size_t)(K + 4) * 8 * npairs; }


size_t bidir_lds_bytes(int K, int nb) {
  return (size_t)((K / nb + TD_BIDIR_CW - 1) / TD_BIDIR_CW + 1) * 2 * 64 * 16;
}

int dec_words_host(int K, int nb) { return nb * ((K / nb + 15) / 16); }

hipError_t launch_load(const TdGroup *dg, int ng, int nblocks, int nb, int sb_input, bool vec,
                       const int16_t *in, size_t in_stride, const int16_t *const *rows,
                       const TdArrays &a, hipStream_t st) {
  if (ng <= 0 || nblocks <= 0) return hipSuccess;
  if (sb_input) {
    if (vec) // 16-byte aligned rows (load_blocks counted 8 elements per thread)
      hipLaunchKernelGGL(k_load_sb8, dim3(nblocks), dim3(256), 0, st, dg, ng, in, in_stride, rows, a);
    else
      hipLaunchKernelGGL(k_load_sb, dim3(nblocks), dim3(256), 0, st, dg, ng, in, in_stride, rows, a);
    return hipGetLastError();
  }
#define LOADNAT(n)                                                                                 \
  do {                                                                                             \
    if (vec)                                                                                       \
      hipLaunchKernelGGL((k_load_nat<n, true>), dim3(nblocks), dim3(256), 0, st, dg, ng, in,        \
                         in_stride, rows, a);                                                      \
    else                                                                                           \
      hipLaunchKernelGGL((k_load_nat<n, false>), dim3(nblocks), dim3(256), 0, st, dg, ng, in,       \
                         in_stride, rows, a);                                                      \
  } while (0)
  if (nb == 32) LOADNAT(32);
  else if (nb == 16) LOADNAT(16);
  else if (nb == 8) LOADNAT(8);
  else if (nb == 1) LOADNAT(1);
  else return hipErrorInvalidValue;
#undef LOADNAT
  return hipGetLastError();
}

hipError_t launch_halfit(int n, int kind, const TdGroup *dg, int ng, int nblocks, size_t lds,
                         bool dec, const TdArrays &arr, const uint8_t *pair_done, hipStream_t st) {
  if (ng <= 0 || nblocks <= 0) return hipSuccess;
  const int mode = (n & 1) ? 1 : (n == 0 ? 2 : 0);
  TdArrays a = arr;
  if (!dec) a.D = nullptr;
#define BIDIR1(nb, div, m, dout, b8)                                                               \
  do {                                                                                             \
    allow_big_lds((const void *)(k_win_bidir<nb, div, m, TD_BIDIR_CW, dout, b8>));                 \
    hipLaunchKernelGGL((k_win_bidir<nb, div, m, TD_BIDIR_CW, dout, b8>), dim3(nblocks), dim3(128), \
                       lds, st, dg, ng, (const s4 *)a.SP0, (s2 *)a.XP1, (s2 *)a.A,               \
                       (uint32_t *)a.D, (const s2 *)a.T, a.plane, pair_done);                                             \
  } while (0)
#define BIDIR(nb, div, m)                                                                          \
  do {                                                                                             \
    if (dec) BIDIR1(nb, div, m, true, false); else BIDIR1(nb, div, m, false, false);               \
  } while (0)
#define BIDIR8(nb, m)                                                                              \
  do {                                                                                             \
    if (dec) BIDIR1(nb, 1, m, true, true); else BIDIR1(nb, 1, m, false, true);                     \
  } while (0)
#define SEQ(kern, m)                                                                               \
  hipLaunchKernelGGL(kern<m>, dim3(nblocks), dim3(64), 0, st, dg, ng, (const s4 *)a.SP0,            \
                     (s2 *)a.XP1, (s2 *)a.A, (uint32_t *)a.D, (const s2 *)a.T, a.plane,             \
                     (s2 *)a.scratch, pair_done)
  switch (kind) {
  case TD_KIND_W16:
    if (mode == 1) BIDIR(16, 0, 1); else if (mode == 2) BIDIR(16, 0, 2); else BIDIR(16, 0, 0);
    break;
  case TD_KIND_W8:
    if (mode == 1) BIDIR(8, 1, 1); else if (mode == 2) BIDIR(8, 1, 2); else BIDIR(8, 1, 0);
    break;
  case TD_KIND_SSE:
    if (mode == 1) SEQ(k_sse_halfit, 1); else if (mode == 2) SEQ(k_sse_halfit, 2); else SEQ(k_sse_halfit, 0);
    break;
  case TD_KIND_GEN:
    if (mode == 1) SEQ(k_gen_halfit, 1); else if (mode == 2) SEQ(k_gen_halfit, 2); else SEQ(k_gen_halfit, 0);
    break;
  case TD_KIND_B16:
  case TD_KIND_B32:
    if (kind == TD_KIND_B16) {
      if (mode == 1) BIDIR8(16, 1); else if (mode == 2) BIDIR8(16, 2); else BIDIR8(16, 0);
    } else {
      if (mode == 1) BIDIR8(32, 1); else if (mode == 2) BIDIR8(32, 2); else BIDIR8(32, 0);
    }
    break;
  default:
    return hipErrorInvalidValue;
  }
#undef SEQ
#undef BIDIR8
#undef BIDIR
#undef BIDIR1
  return hipGetLastError();
}

hipError_t launch_pair_done(const TdGroup *dg, int ng, int npairs, const uint8_t *cb_done,
                            uint8_t *pair_done, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair_done, dim3(nblk(npairs, 256)), dim3(256), 0, st, dg, ng, npairs, cb_done,
                     pair_done);
  return hipGetLastError();
}

hipError_t launch_decide(int n, const TdGroup *dg, int ng, int npairs, const TdArrays &a,
                         uint8_t *outb, size_t out_stride, bool early, uint8_t *cb_done,
                         uint8_t *cb_ok, uint32_t *noi, int max_halfits, uint8_t *pair_done,
                         hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_decide, dim3(npairs), dim3(256), 0, st, n, dg, ng, (const uint32_t *)a.D, outb,
                     out_stride, early ? 1 : 0, cb_done, cb_ok, noi, max_halfits,
                     early ? pair_done : nullptr);
  return hipGetLastError();
}

} // namespace srsgpu

#ifdef TD_TIMING
extern "C" int srsgpu_debug_td_times(unsigned long long *out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(srsgpu::td_times), sizeof(unsigned long long) * n) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
