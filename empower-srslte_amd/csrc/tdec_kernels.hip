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

#include "wave_prio.h"

#include <algorithm>

#include "tdec_kernels.h"

// translation-unit part (see the launchers at the end); the file alone is part 0
#ifndef TD_PART
#define TD_PART 0
#endif

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

// Buffer resources for the windowed decoders' chunk loads and scatter stores. A wave's arrays are
// addressed as (wave base in SGPRs) + (lane's byte offset, loop invariant, VGPR) + (step offset,
// wave-uniform, SGPR): every load and store is one buffer instruction with no per-access VGPR
// address arithmetic, and no VGPR temporaries whose reuse would make the compiler wait for loads
// still in flight (the chunk prefetch of the recursions depends on that).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t mk_rsrc(const void *p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, 0x7FFFFFFF, 0x00020000);
}
typedef uint32_t u4b __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4b bld128(rsrc_t r, uint32_t vo, uint32_t so) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0);
}
__device__ __forceinline__ uint32_t bld32(rsrc_t r, uint32_t vo, uint32_t so) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0);
}
__device__ __forceinline__ void bst32(uint32_t v, rsrc_t r, uint32_t vo) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, vo, 0, 0);
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
// (states 1..7 minus state 0, then state 0 = 0: a literal the next step folds away)
__device__ __forceinline__ void win_norm(int k, St8 &o) {
  if ((k & 1) == 0 && k != 0) {
    s2 z = o.s[0];
#pragma unroll
    for (int i = 1; i < 8; i++) o.s[i] = ssub(o.s[i], z);
    o.s[0] = splat(0);
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
// Windowed decoder (turbodecoder_win.h), two waves per 64 sub-block chains, both starting at
// their end of the sub-block and meeting at M = 16*qm (qm = nc/2 of the nc 16-step chunks):
//   phase 1  wave 0 runs the alpha recursion over chunks 0..qm-1, wave 1 the beta recursion over
//            chunks nc-1..qm; each checkpoints its metric every 16 steps into LDS (alpha: the
//            state entering the chunk; beta: the value the reference stores, before
//            normalisation). One workgroup barrier.
//   phase 2  both waves emit LLRs chunk by chunk, the same way: first the 16 betas of the chunk
//            into registers (wave 0 recomputes them from wave 1's checkpoints, wave 1 continues
//            its own recursion), then the alpha recursion over the chunk with the LLR of every
//            step (wave 0 continues its alpha, wave 1 restarts it from wave 0's checkpoint). The
//            LLR reuses the alpha step's branch sums, so a step of phase 2 costs one beta step and
//            one alpha step plus the LLR, whichever wave runs it.
// Every position is visited with the reference's normalisation schedule, and the integer
// recursions are exact, so every metric equals the reference's. The serial chain is half as
// long as the reference's, and the checkpoints never touch HBM.
static_assert(TD_BIDIR_CW == 16, "phase-2 chunks and decision words hold 16 steps");

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s2 as_s2(uint32_t v) { return __builtin_bit_cast(s2, v); }

// Raw inputs of one group (4 steps of one chain): MODE 1: s0 = X2 (app2), s1 = P1; MODE 0/2:
// s0, s1 = SP0 of steps 0-1 / 2-3 (syst, par0 per step); MODE 0: a = A
template <int MODE> struct Grp {
  u4 s0, s1, a;
};

// x, y and the output operand e of step jj of a group (the input policy of turbodecoder_iter.h
// and win.h:386-393,512-519: DEC1 x = syst (+) app1 saturating, DEC2 x = app2; B8: scaled lanes)
template <int MODE, bool B8>
__device__ __forceinline__ void grp_step(const Grp<MODE> &g, int jj, s2 &x, s2 &y, s2 &e) {
  if (MODE == 1) {
    x = as_s2(g.s0[jj]);
    const s2 p = as_s2(g.s1[jj]);
    y = B8 ? bscale(p) : p;
    e = x;
  } else {
    const u4 &v = jj < 2 ? g.s0 : g.s1;
    const s2 sy = as_s2(v[(jj & 1) * 2]), pa = as_s2(v[(jj & 1) * 2 + 1]);
    const s2 a = MODE == 2 ? splat(0) : as_s2(g.a[jj]);
    if (B8)
      x = MODE == 2 ? bscale(sy) : badd(a, bscale(sy));
    else
      x = MODE == 2 ? sy : sadd(a, sy);
    y = B8 ? bscale(pa) : pa;
    e = a;
  }
}

// a 16-step chunk: 4 groups and, in phase 2, the 16 scatter targets (T16 table words)
template <int MODE> struct Chunk {
  Grp<MODE> g[4];
  u4 t[2];
};
// s_waitcnt vmcnt(0) as a builtin, which the compiler's wait insertion takes into account: a loop
// entered with loads of its first operands still pending gets, at the loop-header merge, waits
// sized for the first iteration in every iteration (there they wait for the previous chunk's
// stores too)
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }
template <int MODE> __device__ __forceinline__ int chunk_t(const Chunk<MODE> &c, int j) {
  return (int)((c.t[j >> 3][(j & 7) >> 1] >> (16 * (j & 1))) & 0xffffu);
}

#ifdef TD_TIMING
// debug build only (make timing): shader-clock stamps per wave of the bidirectional decoder
static __device__ unsigned long long td_times[2048 * 8];
#define TD_T(k)                                                                                    \
  do {                                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) {                                           \
      td_times[(blockIdx.x * 2 + role) * 8 + (k)] = clock64();                                     \
      if ((k) == 0 || (k) == 4) td_times[(blockIdx.x * 2 + role) * 8 + 5 + (k) / 4] = wall_clock64(); \
    }                                                                                              \
  } while (0)
// finer stamps: per chunk of phase 1 (slot q) and per phase-2 chunk (start / betas done / LLRs
// done at 32 + 3 i, i = the i-th chunk the wave emits)
static __device__ unsigned long long td_chunk[2048 * 80];
#define TD_C(k)                                                                                    \
  do {                                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024 && (k) < 80)                                  \
      td_chunk[(blockIdx.x * 2 + role) * 80 + (k)] = clock64();                                    \
    __builtin_amdgcn_sched_barrier(0);                                                             \
  } while (0)
#else
#define TD_T(k)
#define TD_C(k)
#endif

// The body of k_win_bidir: every pointer a __restrict__ parameter, so the scoped no-alias
// facts survive inlining (the group tables would otherwise hide them from the scheduler).
// sp0 / p1 point at the pair's T4 regions, x2 / A at its sub-block-order ones, tbl at the group's
// T16 table.
// Wave-level buffer resources of the windowed decoders: SP0, X2, P1 and A from the wave's first
// pair, the scatter table of the half-iteration; po = byte offset of the lane's pair from the
// wave's first pair in the 4-byte arrays (2 po in SP0).
struct WinRes {
  rsrc_t sp0, x2, p1, a, tb;
  uint32_t po;
};

template <int NB, int DIV, int MODE, bool DOUT, bool B8>
__device__ __forceinline__ void win_bidir_body(const s4 *__restrict__ sp0, s2 *__restrict__ x2,
                                               const s2 *__restrict__ p1, s2 *__restrict__ A,
                                               uint32_t *__restrict__ D, const s2 *__restrict__ tl,
                                               const WinRes &R, s4 *__restrict__ cks, int K, int d,
                                               int role, int lane) {
  constexpr int CW = 16;
  const int L = K / NB;
  const int G4 = (L + 3) >> 2; // T4 groups per chain
  const int nc = (L + CW - 1) / CW;
  const int qm = nc / 2; // meeting chunk: M = CW*qm
  const int tail_xoff = MODE == 1 ? 6 : 0;
  const int K32 = K & ~31; // B8: srslte_vec_sub_bbb saturates below, wraps above (AVX2 body)
  const int G16 = (L + 15) / 16;

  // ---- arithmetic of the variant: 16-bit windows (saturating int16, state-0 normalisation every
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
  // win.h:255-258: states 1..7 minus state 0, state 0 set to 0 (a literal, so the next step's
  // operations on it fold away)
  auto norm0 = [&](St8 &o) {
    const s2 z = o.s[0];
#pragma unroll
    for (int i = 1; i < 8; i++) o.s[i] = ssub(o.s[i], z);
    o.s[0] = splat(0);
  };
  // alpha after step k = CW q + j (win.h:579: k even and k != 0; B8: every k != 0)
  auto nrm_fwd = [&](St8 &o, int q, int j) {
    if (B8) {
      if (!(q == 0 && j == 0)) b_norm_max(o);
    } else if ((j & 1) == 0) {
      if (j != 0)
        norm0(o);
      else if (q != 0)
        norm0(o);
    }
  };
  // beta after a step k != 0 that is even when `even` (win.h:432)
  auto nrm_k = [&](St8 &o, bool even) {
    if (B8)
      b_norm_max(o);
    else if (even)
      norm0(o);
  };

  // ---- checkpoints in LDS: [slot][half][lane] x 16 B (conflict-free b128 accesses)
  auto ck_put = [&](int slot, const St8 &o) {
#ifdef TD_EXP_HALFLDS
    slot >>= 1; // timing experiment only (wrong results): half the checkpoint slots, aliased
#endif
    s4 *p = &cks[((slot * 2) * 64 + lane) * 2];
    p[0] = s4{o.s[0].x, o.s[0].y, o.s[1].x, o.s[1].y};
    p[1] = s4{o.s[2].x, o.s[2].y, o.s[3].x, o.s[3].y};
    s4 *q = &cks[((slot * 2 + 1) * 64 + lane) * 2];
    q[0] = s4{o.s[4].x, o.s[4].y, o.s[5].x, o.s[5].y};
    q[1] = s4{o.s[6].x, o.s[6].y, o.s[7].x, o.s[7].y};
  };
  auto ck_get = [&](int slot, St8 &o) {
#ifdef TD_EXP_HALFLDS
    slot >>= 1;
#endif
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

  // ---- group loads: group g (steps 4g..4g+3) of chain dd, as buffer loads: lane offset (pair,
  // chain) in a VGPR, step offset wave-uniform. SP0 (T4) groups are 32 B (two 16-byte loads), P1
  // (T4) 16 B; X2 and A in sub-block order (4 element loads, one per step).
  auto ld_sb4 = [&](rsrc_t r, int g, int dd) {
    const uint32_t vo = R.po + 4u * (uint32_t)dd, so = 16u * NB * (uint32_t)g;
    return u4{bld32(r, vo, so), bld32(r, vo, so + 4 * NB), bld32(r, vo, so + 8 * NB),
              bld32(r, vo, so + 12 * NB)};
  };
  auto ld_grp = [&](Grp<MODE> &r, int g, int dd) {
#ifdef TD_EXP_L2
    g &= 3; // timing experiment only: every load from the pair's first 4 groups (cache resident)
#endif
    if (MODE == 1) {
      r.s0 = ld_sb4(R.x2, g, dd);
      r.s1 = bld128(R.p1, R.po + 16u * (uint32_t)dd, 16u * NB * (uint32_t)g);
    } else {
      const uint32_t vo = 2u * R.po + 32u * (uint32_t)dd, so = 32u * NB * (uint32_t)g;
      r.s0 = bld128(R.sp0, vo, so);
      r.s1 = bld128(R.sp0, vo, so + 16);
      if (MODE == 0) r.a = ld_sb4(R.a, g, dd);
    }
  };
  // chunk q of this lane's chain: groups 4q..4q+3 (clamped into the chain for the last, partial
  // chunk: the recursion never reads its steps past L); tables only where phase 2 needs them
  auto ld_chunk = [&](Chunk<MODE> &c, int q, bool with_t) {
    const int g0 = 4 * q;
#pragma unroll
    for (int u = 0; u < 4; u++) ld_grp(c.g[u], min(g0 + u, G4 - 1), d); // uniform (SALU) clamp
    if (with_t) {
      const uint32_t vo = 32u * (uint32_t)d, so = 32u * NB * (uint32_t)q;
      c.t[0] = bld128(R.tb, vo, so);
      c.t[1] = bld128(R.tb, vo, so + 16);
    }
    // keep the loads here, a chunk ahead of their use: left alone, the scheduler sinks them
    // towards the first use to save registers, and the waves then wait on memory every chunk
    __builtin_amdgcn_sched_barrier(0);
  };
  auto cstep = [&](const Chunk<MODE> &c, int j, s2 &x, s2 &y, s2 &e) {
    grp_step<MODE, B8>(c.g[j >> 2], j & 3, x, y, e);
  };

  // ---- phase 2 pieces, shared by both waves
  // bst[j] = beta[s0+1+j] for j < n, from `top` = beta[s0+n] before normalisation (normalised
  // first unless it is beta[L]); returns the running beta ready for step s0 (normalised when
  // s0+1 is even... i.e. as the reference leaves it after beta[s0+1])
  auto betas = [&](const Chunk<MODE> &c, St8 top, bool top_is_L, int n, St8 bst[CW]) -> St8 {
    St8 run = top;
#pragma unroll
    for (int j = CW - 1; j >= 0; j--)
      if (j == n - 1) bst[j] = run;
    if (!top_is_L) nrm_k(run, true); // s0 + CW: even, non-zero
#pragma unroll
    for (int j = CW - 2; j >= 0; j--) {
      if (j <= n - 2) {
        s2 x, y, e;
        cstep(c, j + 1, x, y, e);
        bstep(run, x, y);
        bst[j] = run;
        nrm_k(run, ((j + 1) & 1) == 0); // k = s0+1+j >= 1
      }
    }
    return run;
  };
  // alpha recursion over the chunk's n steps from `o` = alpha[s0], with the LLR of every step
  auto alpha_llr = [&](const Chunk<MODE> &c, St8 &o, const St8 bst[CW], int q, int n) {
    const int s0 = CW * q;
    uint32_t dacc = 0;
#pragma unroll
    for (int j = 0; j < CW; j++) {
      if (j < n) {
        s2 x, y, e;
        cstep(c, j, x, y, e);
        s2 mb[8], nw[8];
        if (B8)
          b_alpha_branches(o, x, y, mb, nw);
        else
          win_alpha_branches(o, x, y, mb, nw);
        // max over the 8 branches as a tree (max is exact, so any order is the reference's)
        const St8 &be = bst[j];
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
        {
#ifdef TD_EXP_FIXST
          const int t = chunk_t(c, j) & 15; // timing experiment only: stores stay in one segment
#else
          const int t = chunk_t(c, j); // sub-block index of the scatter target
#endif
          s2 out;
          if (B8) { // ext - app with the reference's saturate / wrap split (K32, see above)
            // the reference's array index decides: j for DEC1, fwd[j] for DEC2
            const bool sat = (MODE == 1 ? t : (s0 + j) * NB + d) < K32;
            out = MODE == 2 ? v : (sat ? bsub(v, e) : wsub(v, e));
          } else {
            out = wsub(v, e); // store_out: DEC1 E' = L - A into app2, DEC2 L - app2 into A
          }
#ifdef TD_EXP_NOX2
          if (MODE != 2) // timing experiment only (wrong results): the first DEC1 stores no X2
#endif
          bst32(__builtin_bit_cast(uint32_t, out), MODE == 1 ? R.a : R.x2, R.po + 4u * (uint32_t)t);
        }
        if (DOUT) dacc |= dec_bits(v) << j;
#pragma unroll
        for (int i = 0; i < 8; i++) o.s[i] = B8 ? bmask(smax(mb[i], nw[i])) : smax(mb[i], nw[i]);
        nrm_fwd(o, q, j);
      }
    }
    if (DOUT) D[d * G16 + q] = dacc;
  };

  St8 o;
  if (role == 0) {
    // ================= forward wave =================
    Chunk<MODE> c0, c1, c2; // phase 1's chunk buffers, the first two loading during the prepass
    {
      // win.h:501-506,512-584 (loop_len = 40) over the last 40 steps of sub-block d-1;
      // move_left (:469-495); sub-block 0 starts in state 0 (:496-500)
      const int dp = d > 0 ? d - 1 : 0;
      st_fill(o, B8 ? 0 : -TD_INF, B8 ? 0 : -TD_INF);
      if ((L & 3) == 0) {
        // ten T4 groups, all loads issued up front
        Grp<MODE> pg[10];
        const int gp = (L - TD_OVERLAP) >> 2;
#pragma unroll
        for (int u = 0; u < 10; u++) ld_grp(pg[u], gp + u, dp);
        ld_chunk(c0, 0, false);
        ld_chunk(c1, min(1, qm - 1), false);
#pragma unroll
        for (int k = 0; k < TD_OVERLAP; k++) {
          s2 x, y, e;
          grp_step<MODE, B8>(pg[k >> 2], k & 3, x, y, e);
          astep(o, x, y);
          pnorm(k, o);
        }
      } else {
        // steps of one chain do not fill T4 groups evenly: element loads, 8 steps at a time
        ld_chunk(c0, 0, false);
        ld_chunk(c1, min(1, qm - 1), false);
        for (int k0 = 0; k0 < TD_OVERLAP; k0 += 8) {
          s2 xs[8], ys[8];
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const int k = L - TD_OVERLAP + k0 + u;
            const int pos = ((k >> 2) * NB + dp) * 4 + (k & 3), sb = k * NB + dp;
            if (MODE == 1) {
              xs[u] = x2[sb];
              const s2 p = p1[pos];
              ys[u] = B8 ? bscale(p) : p;
            } else {
              const s4 v = sp0[pos];
              const s2 a = MODE == 2 ? splat(0) : A[sb];
              if (B8)
                xs[u] = MODE == 2 ? bscale(lo2(v)) : badd(a, bscale(lo2(v)));
              else
                xs[u] = MODE == 2 ? lo2(v) : sadd(a, lo2(v));
              ys[u] = B8 ? bscale(hi2(v)) : hi2(v);
            }
          }
#pragma unroll
          for (int u = 0; u < 8; u++) {
            astep(o, xs[u], ys[u]);
            pnorm(k0 + u, o);
          }
        }
      }
      if (d == 0) st_fill(o, 0, B8 ? 0 : -TD_INF);
    }
    TD_T(1);
    // phase 1: chunks 0 .. qm-1, checkpoint the entering state of each; loads two chunks ahead
    {
      auto fwd_chunk = [&](const Chunk<MODE> &c, int q) {
        TD_C(q);
        ck_put(q, o);
#pragma unroll
        for (int j = 0; j < CW; j++) {
          s2 x, y, e;
          cstep(c, j, x, y, e);
          astep(o, x, y);
          nrm_fwd(o, q, j);
        }
      };
      int q = 0;
      for (; q + 2 < qm; q += 3) {
        ld_chunk(c2, q + 2, false);
        fwd_chunk(c0, q);
        ld_chunk(c0, min(q + 3, qm - 1), false); // unconditional: a load under a branch makes
        fwd_chunk(c1, q + 1);                    // the vmcnt merge wait for the fresh loads
        ld_chunk(c1, min(q + 4, qm - 1), false);
        fwd_chunk(c2, q + 2);
      }
      if (q < qm) fwd_chunk(c0, q);
      if (q + 1 < qm) fwd_chunk(c1, q + 1);
    }
    Chunk<MODE> cur, cnx;
    ld_chunk(cur, qm, true); // phase 2's first chunk, loading across the barrier
    TD_T(2);
    __syncthreads();
    vm_drain();
    TD_T(3);
#ifdef TD_EXP_P1ONLY
    if (K > 0) return; // timing experiment only: prepass and phase 1
#endif
    // phase 2: chunks qm .. nc-1, betas recomputed from the backward wave's checkpoints. One
    // chunk per loop iteration (the next one loading meanwhile); the last chunk, when L is not a
    // multiple of 16, after the loop.
    {
      auto seg = [&](const Chunk<MODE> &c, int q) {
        St8 top, bst[CW];
        TD_C(32 + 3 * (q - qm));
        ck_get(q + 1, top); // beta[CW(q+1)] (beta[L] when q + 1 == nc)
        (void)betas(c, top, q == nc - 1, CW, bst);
        TD_C(33 + 3 * (q - qm));
        alpha_llr(c, o, bst, q, CW);
        TD_C(34 + 3 * (q - qm));
      };
      const int qf = L / CW; // full chunks
      // two chunks per iteration, the buffers alternating (no copies); an odd count first takes
      // one chunk and a single copy, so the loop is entered as it loops
      int q = qm;
      if ((qf - qm) & 1) {
        ld_chunk(cnx, min(q + 1, nc - 1), true);
        seg(cur, q);
        cur = cnx;
        q++;
      }
      for (; q + 1 < qf; q += 2) {
        ld_chunk(cnx, q + 1, true);
        seg(cur, q);
        ld_chunk(cur, min(q + 2, nc - 1), true);
        seg(cnx, q + 1);
      }
      if (qf < nc) {
        // the partial chunk, n = L - CW qf steps (cur holds it): betas by selects, so every
        // metric stays in a register whatever n is; the alpha / LLR steps under uniform guards
        const int q = qf, n = L - CW * qf;
        St8 top, bst[CW];
        ck_get(nc, top); // beta[L], never normalised
        St8 run = top;
        bst[CW - 1] = top;
#pragma unroll
        for (int j = CW - 2; j >= 0; j--) {
          St8 nx = run; // beta[s0+2+j] once j + 1 <= n - 1
          if (B8 || (j & 1) == 0) { // k = s0+2+j even (16-bit) / any (B8); not beta[L]
            St8 nn = nx;
            nrm_k(nn, true);
            const bool is_top = j + 1 == n - 1;
#pragma unroll
            for (int i = 0; i < 8; i++) nx.s[i] = is_top ? nx.s[i] : nn.s[i];
          }
          s2 x, y, e;
          cstep(cur, j + 1, x, y, e);
          bstep(nx, x, y);
          const bool above = j >= n - 1;
#pragma unroll
          for (int i = 0; i < 8; i++) run.s[i] = above ? top.s[i] : nx.s[i];
          bst[j] = run;
        }
        alpha_llr(cur, o, bst, q, n);
      }
    }
  } else {
    // ================= backward wave =================
    Chunk<MODE> c0, c1, c2; // phase 1's chunk buffers, the first two loading during the prepass
    const int qt = nc - 1;  // top chunk, possibly partial; qm < qt (L > 40: nc >= 3)
    {
      // win.h:376-384,386-433 (loop_len = 40) over the first 40 steps of sub-block d+1;
      // move_right (:333-366); the last sub-block starts from the tail trellis (:350-355)
      const int dn = d + 1 < NB ? d + 1 : d;
      st_fill(o, B8 ? 0 : -TD_INF, B8 ? 0 : -TD_INF);
      Grp<MODE> pg[10];
#pragma unroll
      for (int u = 0; u < 10; u++) ld_grp(pg[u], u, dn);
      s2 tv[6]; // this decoder's tail values (x, y) x 3
#pragma unroll
      for (int u = 0; u < 6; u++) tv[u] = tl[tail_xoff + u];
      ld_chunk(c0, qt, false);
      ld_chunk(c1, qt - 1, false); // qt - 1 >= qm
#pragma unroll
      for (int k = TD_OVERLAP - 1; k >= 0; k--) {
        s2 x, y, e;
        grp_step<MODE, B8>(pg[k >> 2], k & 3, x, y, e);
        bstep(o, x, y);
        pnorm(k, o);
      }
      St8 t;
      if (B8)
        b_tail_trellis(tv, 0, t);
      else
        win_tail_trellis(tv, 0, t);
      if (d == NB - 1) o = t;
    }
    ck_put(nc, o); // beta[L] (win.h:372-374)
    TD_T(1);
    // phase 1: chunks nc-1 .. qm (steps L-1 .. M); bpre ends as beta[M] before normalisation
    St8 bpre;
    {
      // the state before normalisation at step CW q goes to slot q: a beta checkpoint for q > qm,
      // bpre for q == qm (slot qm is free: alpha checkpoints fill 0..qm-1, beta ones qm+1..nc),
      // read back after the loop, so the loop body has no branch on q
      auto bwd_chunk = [&](const Chunk<MODE> &c, int q, int n) { // q > 0: norm never at 0
        TD_C(nc - 1 - q);
#pragma unroll
        for (int j = CW - 1; j >= 0; j--) {
          if (j < n) {
            s2 x, y, e;
            cstep(c, j, x, y, e);
            bstep(o, x, y);
            if (j == 0) ck_put(q, o);
            nrm_k(o, (j & 1) == 0);
          }
        }
      };
      ld_chunk(c2, max(qt - 2, qm), false);
      bwd_chunk(c0, qt, L - CW * qt);
      // then full chunks q, q-1, q-2 in c1, c2, c0 (rotating), down to qm; loads two ahead
      int q = qt - 1;
      for (; q - 2 >= qm; q -= 3) {
        ld_chunk(c0, q - 2, false);
        bwd_chunk(c1, q, CW);
        ld_chunk(c1, max(q - 3, qm), false);
        bwd_chunk(c2, q - 1, CW);
        ld_chunk(c2, max(q - 4, qm), false);
        bwd_chunk(c0, q - 2, CW);
      }
      if (q >= qm) bwd_chunk(c1, q, CW);
      if (q - 1 >= qm) bwd_chunk(c2, q - 1, CW);
      ck_get(qm, bpre); // beta[M] before normalisation
    }
    Chunk<MODE> cur, cnx;
    ld_chunk(cur, qm - 1, true); // phase 2's first chunk, loading across the barrier
    TD_T(2);
    __syncthreads();
    vm_drain();
    TD_T(3);
#ifdef TD_EXP_P1ONLY
    if (K > 0) return; // timing experiment only: prepass and phase 1
#endif
    // phase 2: chunks qm-1 .. 0 (full), one per loop iteration: the beta recursion continues,
    // alphas restart from the forward wave's checkpoints
    {
      auto seg = [&](const Chunk<MODE> &c, int q) {
        St8 bst[CW];
        TD_C(32 + 3 * (qm - 1 - q));
        St8 run = betas(c, bpre, false, CW, bst);
        if (q > 0) { // beta[s0] before normalisation, the next chunk's top
          s2 x, y, e;
          cstep(c, 0, x, y, e);
          bstep(run, x, y);
          bpre = run;
        }
        St8 a;
        ck_get(q, a);
        TD_C(33 + 3 * (qm - 1 - q));
        alpha_llr(c, a, bst, q, CW);
        TD_C(34 + 3 * (qm - 1 - q));
      };
      int q = qm - 1; // two chunks per iteration, as in the forward wave
      if (qm & 1) {
        ld_chunk(cnx, max(q - 1, 0), true);
        seg(cur, q);
        cur = cnx;
        q--;
      }
      for (; q >= 1; q -= 2) {
        ld_chunk(cnx, q - 1, true);
        seg(cur, q);
        ld_chunk(cur, max(q - 2, 0), true);
        seg(cnx, q - 1);
      }
    }
  }
}

// the wave's buffer resources (WinRes): bases at the wave's first pair pw, lane offset of `pair`
template <int NB>
__device__ __forceinline__ WinRes win_res(const TdGroup &G, int K, int blk, int pair, const s4 *SP0,
                                          s2 *XP1, s2 *Aarr, size_t plane, const uint16_t *tb) {
  const int pe = t4_pair_elems(K, NB);
  const int pw = (blk * 64) / NB;
  const size_t wb = (size_t)G.elem0 + (size_t)pw * pe;
  WinRes R;
  R.sp0 = mk_rsrc(SP0 + wb);
  R.x2 = mk_rsrc(XP1 + wb);
  R.p1 = mk_rsrc(XP1 + plane + wb);
  R.a = mk_rsrc(Aarr + wb);
  R.tb = mk_rsrc(tb);
  R.po = (uint32_t)((pair - pw) * pe) * 4u;
  return R;
}

#ifndef TD_BIDIR_WAVES
#define TD_BIDIR_WAVES 1 // minimum waves per SIMD the windowed decoders are compiled for
#endif
#ifndef TD_H0_WAVES
#define TD_H0_WAVES TD_BIDIR_WAVES // the same for the first half-iteration (MODE 2) alone
#endif
template <int NB, int DIV, int MODE, int CW, bool DOUT, bool B8>
__global__ __launch_bounds__(128, MODE == 2 ? TD_H0_WAVES : TD_BIDIR_WAVES) void k_win_bidir(const TdGroup *__restrict__ groups, int ngroups,
                                                   const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                   s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                   const s2 *__restrict__ T, size_t plane,
                                                   const uint8_t *__restrict__ pair_done, int prio) {
  // checkpoint slots in (dynamic) LDS, [slot][half][lane] x 16 B (conflict-free b128 accesses);
  // nc + 1 slots of 2 KiB: 50 KiB at K = 6144 with 16 sub-blocks
  extern __shared__ s4 cks[];
  wave_prio(prio);
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); // 0: alpha, 1: beta
  TD_T(0);
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int K = G.K, npairs = G.npairs;
  const int blk = blockIdx.x - G.blk_half;
  const int lane = threadIdx.x & 63;
  const int gl = blk * 64 + lane;
  const int nlanes = npairs * NB;
  // lanes past the group's chains repeat the last chain: same inputs, same results, stored to
  // the same addresses (stores are unconditional: a per-lane guard costs a branch per step)
  const int g = gl < nlanes ? gl : nlanes - 1;
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
  // pairs already finished (early stop) in a partly finished workgroup decode on: their arrays
  // and decision words are never read again (k_decide skips them)
  const size_t base = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, NB);
  const s4 *sp0 = SP0 + base;
  s2 *xp1 = XP1 + base;              // app2 (DEC1 output)
  const s2 *p1 = XP1 + plane + base; // par1
  s2 *A = Aarr + base;
  uint32_t *D = DOUT ? Darr + G.dw0 + (size_t)pair * dec_words(K, NB) : nullptr;
  const s2 *tl = T + (size_t)(G.pair0 + pair) * 12;
  const WinRes R = win_res<NB>(G, K, blk, pair, SP0, XP1, Aarr, plane, MODE == 1 ? G.fwd : G.rev);
  win_bidir_body<NB, DIV, MODE, DOUT, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
  TD_T(4);
}

// ------------------------------------------------------------------ windowed, spread (latency) ----
// One half-iteration of a FEW pairs (the drop-in srslte_tdec_iteration: one code block per call),
// where k_win_bidir leaves the chip idle and its serial chain (the prepass, then half the chunks of
// one recursion, then the other half with the LLR, ~100 packed ops a step) is the call's latency.
// Here a workgroup of TD_SPREAD_THREADS holds ONE pair:
//   phase A  wave 0 runs the whole alpha recursion (prepass + chunks 0..nc-1) and checkpoints the
//            state entering every chunk, wave 1 the whole beta recursion (prepass, tail, chunks
//            nc-1..1) and checkpoints beta at every chunk boundary (the value before
//            normalisation, as k_win_bidir's backward wave does); ~24 ops a step
//   phase B  every (chain d, chunk q) is an independent task (K / 16 of them): betas recomputed
//            from the checkpoint above the chunk, the alpha recursion with the LLR from the one
//            below it — the pieces k_win_bidir's phase 2 runs, spread over every lane of the
//            workgroup instead of one lane per chain.
// The serial chain becomes L + 40 steps of one recursion plus two chunk tasks. Same steps, same
// normalisation schedule and same checkpoint values as k_win_bidir, so the output is identical
// (tests: every batch of one pair goes through here, larger ones through k_win_bidir).
// Needs L = K / NB a multiple of 16 (no partial chunk) and nc >= 3 (spread_ok).
// quad_perm DPP move (within each group of 4 lanes)
template <int CTRL> __device__ __forceinline__ uint32_t dppq(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
#ifdef TD_TIMING
#define SP_T(k)                                                                                    \
  do {                                                                                             \
    if (lane == 0 && blockIdx.x < 1024) td_times[blockIdx.x * 8 + (k)] = clock64();                \
  } while (0)
#else
#define SP_T(k)
#endif
#define TD_SPREAD_THREADS 512
#ifndef TD_SPREAD_SPLIT
#define TD_SPREAD_SPLIT 1 // workgroups per pair: phase A on each, phase B's tasks shared (r06_s30: 2 was
                          // slower: the arrival counter, fences and decision-word reload before the bytes
                          // cost more than the halved phase B)
#endif
#define TD_SPREAD_MAX_PAIRS 16 // at most this many pairs per job: k_win_bidir beyond

template <int NB, int DIV, int MODE, bool DOUT, bool B8>
__global__ __launch_bounds__(TD_SPREAD_THREADS) void k_win_spread(const TdGroup *__restrict__ groups,
                                                                const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                                s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                                const s2 *__restrict__ T, size_t plane,
                                                                const uint8_t *__restrict__ pair_done,
                                                                uint8_t *__restrict__ outb, size_t out_stride,
                                                                uint32_t *__restrict__ cnt, uint32_t *__restrict__ flag,
                                                                uint32_t seq) {
  constexpr int CW = 16;
  extern __shared__ s4 spk[]; // checkpoints [slot][chain] x 32 B: alpha 0..nc-1, beta nc..2nc
  __shared__ uint32_t sdw[6144 / 16]; // the decision words again, for the fused bytes (outb)
  const TdGroup &G = groups[0];
  const int K = G.K, pair = blockIdx.x / TD_SPREAD_SPLIT, part = blockIdx.x % TD_SPREAD_SPLIT;
  if (pair_done && pair_done[G.pair0 + pair]) return; // uniform over the workgroup
  const int L = K / NB, nc = L / CW;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (wave == 0) SP_T(0);
  const int pe = t4_pair_elems(K, NB);
  const size_t base = (size_t)G.elem0 + (size_t)pair * pe;
  WinRes R;
  R.sp0 = mk_rsrc(SP0 + base);
  R.x2 = mk_rsrc(XP1 + base);
  R.p1 = mk_rsrc(XP1 + plane + base);
  R.a = mk_rsrc(Aarr + base);
  R.tb = mk_rsrc(MODE == 1 ? G.fwd : G.rev);
  R.po = 0;
  uint32_t *D = DOUT ? Darr + G.dw0 + (size_t)pair * dec_words(K, NB) : nullptr;
  const s2 *tl = T + (size_t)(G.pair0 + pair) * 12;
  const int K32 = K & ~31;

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
  auto norm0 = [&](St8 &o) {
    const s2 z = o.s[0];
#pragma unroll
    for (int i = 1; i < 8; i++) o.s[i] = ssub(o.s[i], z);
    o.s[0] = splat(0);
  };
  auto nrm_fwd = [&](St8 &o, int q, int j) { // as win_bidir_body's
    if (B8) {
      if (!(q == 0 && j == 0)) b_norm_max(o);
    } else if ((j & 1) == 0) {
      if (j != 0 || q != 0) norm0(o);
    }
  };
  auto nrm_k = [&](St8 &o, bool even) {
    if (B8)
      b_norm_max(o);
    else if (even)
      norm0(o);
  };
  auto pnorm = [&](int k, St8 &o) {
    if (B8)
      b_norm(k, o);
    else
      win_norm(k, o);
  };
  auto ck_put = [&](int slot, int d, const St8 &o) {
    s4 *p = &spk[(slot * NB + d) * 4];
#pragma unroll
    for (int i = 0; i < 4; i++) p[i] = s4{o.s[2 * i].x, o.s[2 * i].y, o.s[2 * i + 1].x, o.s[2 * i + 1].y};
  };
  auto ck_get = [&](int slot, int d, St8 &o) {
    const s4 *p = &spk[(slot * NB + d) * 4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const s4 v = p[i];
      o.s[2 * i] = lo2(v);
      o.s[2 * i + 1] = hi2(v);
    }
  };
  // group g of chain dd; `lo` = per-lane byte offset added to the wave-uniform step offset (phase B:
  // the lane's chunk), as in win_bidir_body's loads
  auto ld_sb4 = [&](rsrc_t r, int g, int dd, uint32_t lo) {
    const uint32_t vo = 4u * (uint32_t)dd + lo, so = 16u * NB * (uint32_t)g;
    return u4{bld32(r, vo, so), bld32(r, vo, so + 4 * NB), bld32(r, vo, so + 8 * NB),
              bld32(r, vo, so + 12 * NB)};
  };
  auto ld_grp = [&](Grp<MODE> &r, int g, int dd, uint32_t lo) {
    if (MODE == 1) {
      r.s0 = ld_sb4(R.x2, g, dd, lo);
      r.s1 = bld128(R.p1, 16u * (uint32_t)dd + lo, 16u * NB * (uint32_t)g);
    } else {
      const uint32_t vo = 32u * (uint32_t)dd + 2u * lo, so = 32u * NB * (uint32_t)g;
      r.s0 = bld128(R.sp0, vo, so);
      r.s1 = bld128(R.sp0, vo, so + 16);
      if (MODE == 0) r.a = ld_sb4(R.a, g, dd, lo);
    }
  };
  auto ld_chunk = [&](Chunk<MODE> &c, int q, int dd) { // phase A: q wave-uniform
#ifdef TD_EXP_SPREAD_L2
    q &= 1; // timing experiment only (wrong results): phase A's chunk loads from two cache-resident chunks
#endif
#pragma unroll
    for (int u = 0; u < 4; u++) ld_grp(c.g[u], 4 * q + u, dd, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto cstep = [&](const Chunk<MODE> &c, int j, s2 &x, s2 &y, s2 &e) {
    grp_step<MODE, B8>(c.g[j >> 2], j & 3, x, y, e);
  };

  if (!B8 && wave < 4) {
    // ---- phase A, 16-bit windows, state-parallel: a quad of lanes per chain and block (wave 0 / 2:
    // alpha of the pair's block 0 / 1, wave 1 / 3: beta), each lane two states in one packed
    // register. The trellis is four butterflies: alpha lane r holds (a[2r], a[2r+1]) and forms
    // (a'[r], a'[r+4]); beta lane r holds (b[r], b[r+4]) and forms (b'[2r], b'[2r+1]). A step is one
    // add on the lane's pair, one on the swapped pair, one max, and two quad permutes (DPP) plus a
    // byte permute to bring the next step's pair in — the same saturating sums and maxima as
    // win_alpha_step / win_beta_step, state by state, so every metric is the reference's.
    const int role = wave & 1, h = wave >> 1;
    const int d = (lane >> 2) % NB, r = lane & 3;
    // per-lane branch metrics: g = (gP, gQ): lane 0 (0, xy), 1 (x, y), 2 (y, x), 3 (xy, 0), the
    // same table for both recursions (gP added to the lane's pair, gQ to the swapped pair)
    // as byte selections of block h's x / y (or zero: selector 0x0C) into the two halves
    const uint32_t hb = h ? 0x0302u : 0x0100u, zb = 0x0C0Cu;
    const uint32_t SX = ((r == 1 || r == 3) ? hb : zb) | (((r == 0 || r == 2) ? hb : zb) << 16);
    const uint32_t SY = ((r == 2 || r == 3) ? hb : zb) | (((r == 0 || r == 1) ? hb : zb) << 16);
    const uint32_t asel = r < 2 ? 0x05040100u : 0x07060302u, bsel = (r & 1) ? 0x07060302u : 0x05040100u;
    auto bits = [](s2 v) { return __builtin_bit_cast(uint32_t, v); };
    auto bfly = [&](uint32_t v, s2 x, s2 y) -> uint32_t { // (P, Q) maxima of the lane's butterfly
      const s2 g = sadd(as_s2(__builtin_amdgcn_perm(bits(x), bits(x), SX)),
                        as_s2(__builtin_amdgcn_perm(bits(y), bits(y), SY)));
      const s2 vv = as_s2(v);
      return bits(smax(sadd(vv, s2{g.x, g.x}), sadd(s2{vv.y, vv.x}, s2{g.y, g.y})));
    };
    // nrm: the step's normalisation (win.h:255-258: minus the new state 0, which is lane 0's low
    // half of the butterfly output in both layouts), its broadcast beside the redistribution
    auto qa = [&](uint32_t &v, s2 x, s2 y, bool nrm) { // alpha: (a'[r], a'[r+4]) -> (a'[2r], a'[2r+1])
      const uint32_t w = bfly(v, x, y);
      const s2 z = as_s2(dppq<0x00>(w));
      v = __builtin_amdgcn_perm(dppq<0xDD>(w), dppq<0x88>(w), asel); // quad_perm [1,3,1,3], [0,2,0,2]
      if (nrm) v = bits(ssub(as_s2(v), s2{z.x, z.x}));
    };
    auto qb = [&](uint32_t &u, s2 x, s2 y, bool nrm) { // beta: (b'[2r], b'[2r+1]) -> (b'[r], b'[r+4])
      const uint32_t w = bfly(u, x, y);
      const s2 z = as_s2(dppq<0x00>(w));
      u = __builtin_amdgcn_perm(dppq<0xFA>(w), dppq<0x50>(w), bsel); // quad_perm [2,2,3,3], [0,0,1,1]
      if (nrm) u = bits(ssub(as_s2(u), s2{z.x, z.x}));
    };
    short *ck16 = reinterpret_cast<short *>(spk);
    auto ck_at = [&](int slot, int s) -> short & { // state s of block h in slot `slot`, chain d
      return ck16[(slot * NB + d) * 16 + 4 * (s >> 1) + 2 * (s & 1) + h];
    };
    const uint32_t NEG = 0xffffu & (uint32_t)(uint16_t)(short)-TD_INF;
    uint32_t v = NEG | (NEG << 16);
    Chunk<MODE> c0, c1, c2;
    if (role == 0) {
      const int dp = d > 0 ? d - 1 : 0;
      {
        Grp<MODE> pg[10];
        const int gp = (L - TD_OVERLAP) >> 2;
#pragma unroll
        for (int u = 0; u < 10; u++) ld_grp(pg[u], gp + u, dp, 0);
        ld_chunk(c0, 0, d);
        ld_chunk(c1, 1, d);
#pragma unroll
        for (int k = 0; k < TD_OVERLAP; k++) {
          s2 x, y, e;
          grp_step<MODE, false>(pg[k >> 2], k & 3, x, y, e);
          qa(v, x, y, (k & 1) == 0 && k != 0);
        }
      }
      if (wave == 0) SP_T(1);
      if (d == 0) v = r == 0 ? (NEG << 16) : (NEG | (NEG << 16)); // state 0 = 0 (win.h:496-500)
      auto fwd_chunk = [&](const Chunk<MODE> &c, int q) {
        ck_at(q, 2 * r) = (short)(v & 0xffffu);
        ck_at(q, 2 * r + 1) = (short)(v >> 16);
#pragma unroll
        for (int j = 0; j < CW; j++) {
          s2 x, y, e;
          cstep(c, j, x, y, e);
          qa(v, x, y, (j & 1) == 0 && (j != 0 || q != 0));
        }
      };
      int q = 0;
      for (; q + 2 < nc; q += 3) {
        ld_chunk(c2, q + 2, d);
        fwd_chunk(c0, q);
        ld_chunk(c0, min(q + 3, nc - 1), d);
        fwd_chunk(c1, q + 1);
        ld_chunk(c1, min(q + 4, nc - 1), d);
        fwd_chunk(c2, q + 2);
      }
      if (q < nc) fwd_chunk(c0, q);
      if (q + 1 < nc) fwd_chunk(c1, q + 1);
      if (wave == 0) SP_T(2);
    } else {
      const int dn = d + 1 < NB ? d + 1 : d;
      {
        Grp<MODE> pg[10];
#pragma unroll
        for (int u = 0; u < 10; u++) ld_grp(pg[u], u, dn, 0);
        s2 tv[6];
#pragma unroll
        for (int u = 0; u < 6; u++) tv[u] = tl[(MODE == 1 ? 6 : 0) + u];
        ld_chunk(c0, nc - 1, d);
        ld_chunk(c1, nc - 2, d);
#pragma unroll
        for (int k = TD_OVERLAP - 1; k >= 0; k--) {
          s2 x, y, e;
          grp_step<MODE, false>(pg[k >> 2], k & 3, x, y, e);
          qb(v, x, y, (k & 1) == 0 && k != 0);
        }
        if (d == NB - 1) { // the last chain starts from the tail trellis (win.h:350-355)
          St8 t;
          win_tail_trellis(tv, 0, t);
          s2 lo = t.s[0], hi = t.s[4];
#pragma unroll
          for (int i = 1; i < 4; i++)
            if (r == i) {
              lo = t.s[i];
              hi = t.s[i + 4];
            }
          v = h ? ((uint32_t)(uint16_t)lo.y | ((uint32_t)(uint16_t)hi.y << 16))
                : ((uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)hi.x << 16));
        }
      }
      auto put_b = [&](int slot) {
        ck_at(slot, r) = (short)(v & 0xffffu);
        ck_at(slot, r + 4) = (short)(v >> 16);
      };
      put_b(2 * nc); // beta[L]
      auto bwd_chunk = [&](const Chunk<MODE> &c, int q) { // q >= 1
#pragma unroll
        for (int j = CW - 1; j >= 0; j--) {
          s2 x, y, e;
          cstep(c, j, x, y, e);
          if (j == 0) { // the checkpoint is beta[16 q] before its normalisation
            qb(v, x, y, false);
            put_b(nc + q);
            v = bits(ssub(as_s2(v), s2{as_s2(dppq<0x00>(v)).x, as_s2(dppq<0x00>(v)).x}));
          } else {
            qb(v, x, y, (j & 1) == 0);
          }
        }
      };
      int q = nc - 1;
      for (; q - 2 >= 1; q -= 3) {
        ld_chunk(c2, q - 2, d);
        bwd_chunk(c0, q);
        ld_chunk(c0, max(q - 3, 1), d);
        bwd_chunk(c1, q - 1);
        ld_chunk(c1, max(q - 4, 1), d);
        bwd_chunk(c2, q - 2);
      }
      if (q >= 1) bwd_chunk(c0, q);
      if (q - 1 >= 1) bwd_chunk(c1, q - 1);
      if (wave == 1) SP_T(3);
    }
  } else if (B8 && wave == 0) {
    // ---- phase A, alpha: win.h:501-506,512-584 prepass over the last 40 steps of chain d-1, then
    // every chunk, the entering state checkpointed
    const int d = lane % NB, dp = d > 0 ? d - 1 : 0;
    St8 o;
    st_fill(o, B8 ? 0 : -TD_INF, B8 ? 0 : -TD_INF);
    Chunk<MODE> c0, c1, c2;
    {
      Grp<MODE> pg[10];
      const int gp = (L - TD_OVERLAP) >> 2;
#pragma unroll
      for (int u = 0; u < 10; u++) ld_grp(pg[u], gp + u, dp, 0);
      ld_chunk(c0, 0, d);
      ld_chunk(c1, 1, d);
#pragma unroll
      for (int k = 0; k < TD_OVERLAP; k++) {
        s2 x, y, e;
        grp_step<MODE, B8>(pg[k >> 2], k & 3, x, y, e);
        astep(o, x, y);
        pnorm(k, o);
      }
    }
    if (d == 0) st_fill(o, 0, B8 ? 0 : -TD_INF);
    auto fwd_chunk = [&](const Chunk<MODE> &c, int q) {
      ck_put(q, d, o);
#pragma unroll
      for (int j = 0; j < CW; j++) {
        s2 x, y, e;
        cstep(c, j, x, y, e);
        astep(o, x, y);
        nrm_fwd(o, q, j);
      }
    };
    int q = 0;
    for (; q + 2 < nc; q += 3) {
      ld_chunk(c2, q + 2, d);
      fwd_chunk(c0, q);
      ld_chunk(c0, min(q + 3, nc - 1), d);
      fwd_chunk(c1, q + 1);
      ld_chunk(c1, min(q + 4, nc - 1), d);
      fwd_chunk(c2, q + 2);
    }
    if (q < nc) fwd_chunk(c0, q);
    if (q + 1 < nc) fwd_chunk(c1, q + 1);
  } else if (B8 && wave == 1) {
    // ---- phase A, beta: win.h:376-384,386-433 prepass over the first 40 steps of chain d+1 (the
    // last chain from the tail trellis, :350-355), beta[L] and beta[16 q] for q = nc-1..1
    const int d = lane % NB, dn = d + 1 < NB ? d + 1 : d;
    St8 o;
    st_fill(o, B8 ? 0 : -TD_INF, B8 ? 0 : -TD_INF);
    Chunk<MODE> c0, c1, c2;
    {
      Grp<MODE> pg[10];
#pragma unroll
      for (int u = 0; u < 10; u++) ld_grp(pg[u], u, dn, 0);
      s2 tv[6];
#pragma unroll
      for (int u = 0; u < 6; u++) tv[u] = tl[(MODE == 1 ? 6 : 0) + u];
      ld_chunk(c0, nc - 1, d);
      ld_chunk(c1, nc - 2, d);
#pragma unroll
      for (int k = TD_OVERLAP - 1; k >= 0; k--) {
        s2 x, y, e;
        grp_step<MODE, B8>(pg[k >> 2], k & 3, x, y, e);
        bstep(o, x, y);
        pnorm(k, o);
      }
      St8 t;
      if (B8)
        b_tail_trellis(tv, 0, t);
      else
        win_tail_trellis(tv, 0, t);
      if (d == NB - 1) o = t;
    }
    ck_put(2 * nc, d, o); // beta[L]
    auto bwd_chunk = [&](const Chunk<MODE> &c, int q) { // q >= 1
#pragma unroll
      for (int j = CW - 1; j >= 0; j--) {
        s2 x, y, e;
        cstep(c, j, x, y, e);
        bstep(o, x, y);
        if (j == 0) ck_put(nc + q, d, o);
        nrm_k(o, (j & 1) == 0);
      }
    };
    int q = nc - 1;
    for (; q - 2 >= 1; q -= 3) {
      ld_chunk(c2, q - 2, d);
      bwd_chunk(c0, q);
      ld_chunk(c0, max(q - 3, 1), d);
      bwd_chunk(c1, q - 1);
      ld_chunk(c1, max(q - 4, 1), d);
      bwd_chunk(c2, q - 2);
    }
    if (q >= 1) bwd_chunk(c0, q);
    if (q - 1 >= 1) bwd_chunk(c1, q - 1);
  }
  // ---- phase B's inputs, loaded before the barrier: waves 4.. (idle in phase A) load theirs while
  // phase A runs. The pair's TD_SPREAD_SPLIT workgroups (on as many CUs) each ran phase A and take
  // their share of the tasks, at most one per thread (launch_halfit_spread checks K / 16).
  const int t_lo = part * NB * nc / TD_SPREAD_SPLIT, t_hi = (part + 1) * NB * nc / TD_SPREAD_SPLIT;
  const int t = t_lo + tid, q = t / NB, d = t % NB;
  const bool has = t < t_hi;
  Chunk<MODE> c;
  if (has) {
    const uint32_t lo = 16u * NB * 4u * (uint32_t)q; // 4 T4 groups per chunk, 16 B per group and chain
#pragma unroll
    for (int u = 0; u < 4; u++) ld_grp(c.g[u], u, d, lo);
    const uint32_t vo = 32u * (uint32_t)d + 32u * NB * (uint32_t)q;
    c.t[0] = bld128(R.tb, vo, 0);
    c.t[1] = bld128(R.tb, vo, 16);
  }
  __shared__ uint16_t sdm[6144]; // dmap, for the fused bytes after DEC2 (staged by the idle waves)
  if (MODE == 1 && DOUT && outb && wave >= 4) {
    const gptr_t<uint32_t> dm32 = gptr((const uint32_t *)G.dmap);
    for (int i = tid - 256; i < K / 2; i += TD_SPREAD_THREADS - 256)
      reinterpret_cast<uint32_t *>(sdm)[i] = dm32[i];
  }
  __syncthreads();
  if (wave == 0) SP_T(4);
#ifdef TD_EXP_SPREAD_AONLY
  if (K > 0) return; // timing experiment only (wrong results): phase A alone
#endif

  if (has) {
    // betas of the chunk (win_bidir_body's `betas` with n = CW): bst[j] = beta[16 q + 1 + j]
    St8 run, bst[CW];
    ck_get(nc + q + 1, d, run); // beta[16 (q + 1)] before normalisation (beta[L] for the top chunk)
    bst[CW - 1] = run;
    if (q + 1 < nc) nrm_k(run, true);
#pragma unroll
    for (int j = CW - 2; j >= 0; j--) {
      s2 x, y, e;
      cstep(c, j + 1, x, y, e);
      bstep(run, x, y);
      bst[j] = run;
      nrm_k(run, ((j + 1) & 1) == 0);
    }
    // alpha with the LLR (win_bidir_body's `alpha_llr`, n = CW)
    St8 o;
    ck_get(q, d, o);
    const int s0 = CW * q;
    uint32_t dacc = 0;
#pragma unroll
    for (int j = 0; j < CW; j++) {
      s2 x, y, e;
      cstep(c, j, x, y, e);
      s2 mb[8], nw[8];
      if (B8)
        b_alpha_branches(o, x, y, mb, nw);
      else
        win_alpha_branches(o, x, y, mb, nw);
      const St8 &be = bst[j];
      s2 t0[8], t1[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        t0[i] = sadd(be.s[i], mb[i]);
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
        v = bmask(v >> 1);
      else if (DIV)
        v = v >> 1;
      const int tt = chunk_t(c, j);
      s2 out;
      if (B8) {
        const bool sat = (MODE == 1 ? tt : (s0 + j) * NB + d) < K32;
        out = MODE == 2 ? v : (sat ? bsub(v, e) : wsub(v, e));
      } else {
        out = wsub(v, e);
      }
      bst32(__builtin_bit_cast(uint32_t, out), MODE == 1 ? R.a : R.x2, 4u * (uint32_t)tt);
      if (DOUT) dacc |= dec_bits(v) << j;
#pragma unroll
      for (int i = 0; i < 8; i++) o.s[i] = B8 ? bmask(smax(mb[i], nw[i])) : smax(mb[i], nw[i]);
      nrm_fwd(o, q, j);
    }
    if (DOUT) {
      D[d * nc + q] = dacc;
      sdw[d * nc + q] = dacc;
    }
  }
  // ---- the decision bytes of the pair's blocks (k_decide's fixed-iteration output, fused: the drop-in
  // srslte_tdec_iteration's one launch per call), MSB first (turbodecoder.c:353-360). With L a multiple
  // of 16 the chain-major index of natural position p after DEC1 is p itself; after DEC2 dmap[p].
  if (wave == 0) SP_T(5);
  if (DOUT && outb) {
    if (TD_SPREAD_SPLIT > 1) { // the last of the pair's workgroups to finish writes the bytes
      __shared__ int last;
      __threadfence();
      __syncthreads();
      if (tid == 0) last = atomicAdd(&cnt[pair], 1u) == TD_SPREAD_SPLIT - 1;
      __syncthreads();
      if (!last) return;
      if (tid == 0) cnt[pair] = 0; // for the next launch
      __threadfence();
      for (int i = tid; i < NB * nc; i += TD_SPREAD_THREADS)
        sdw[i] = __hip_atomic_load(&D[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const int nwd = K / 32; // K is a multiple of 16 NB >= 128: whole 32-bit words
    const bool w32 = ((uintptr_t)outb & 3u) == 0 && (out_stride & 3u) == 0;
    for (int i = tid; i < 2 * nwd; i += TD_SPREAD_THREADS) {
      const int h = i >= nwd, w = i - h * nwd, cb = 2 * pair + h;
      if (cb >= G.ncb) continue;
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int p = 32 * w + 8 * j;
        uint32_t v = 0;
        if (MODE != 1) {
          v = (sdw[p >> 4] >> (16 * h + (p & 15))) & 0xffu;
        } else {
#pragma unroll
          for (int b = 0; b < 8; b++) {
            const int c = sdm[p + b];
            v |= ((sdw[c >> 4] >> ((c & 15) + 16 * h)) & 1u) << b;
          }
        }
        word |= (__builtin_bitreverse32(v) >> 24) << (8 * j);
      }
      uint8_t *row = outb + (size_t)(G.cb0 + cb) * out_stride;
      if (w32) {
        reinterpret_cast<uint32_t *>(row)[w] = word;
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++) row[4 * w + j] = (uint8_t)(word >> (8 * j));
      }
    }
    if (flag) { // host-mapped completion word: the caller polls it instead of synchronising the stream
      __threadfence_system();
      __syncthreads();
      if (tid == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (wave == 0) SP_T(6);
  }
}

// Half-iterations n0 .. n0+nh-1 of a fixed-iteration job in ONE launch (turbodecoder.c:510-533,
// srslte_tdec_run_all's loop). A pair's 16 / 8 / 32 chains all sit in one workgroup, and the
// interleaver permutes within a code block, so half-iteration n+1 of a pair reads only what this
// workgroup wrote in half-iteration n: a workgroup barrier orders them (the waves of a workgroup
// share the CU's L1, so workgroup-scope ordering is enough). Compared with one launch per
// half-iteration, the waves never restart together: the start-up burst of every wave's prepass
// loads (all 1024 waves at once, ~10 % of a half-iteration) happens once, and the launch gaps and
// end-of-kernel skew go. Decisions only after the last half-iteration (early stop keeps the
// per-half-iteration launches and k_decide between them). Arithmetic identical to k_win_bidir.
template <int NB, int DIV, bool B8>
__global__ __launch_bounds__(128, TD_BIDIR_WAVES) void k_win_bidir_run(const TdGroup *__restrict__ groups, int ngroups,
                                                       const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                       s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                       const s2 *__restrict__ T, size_t plane, int n0,
                                                       int nh, int dout) {
  extern __shared__ s4 cks[];
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int K_ = G.K, npairs = G.npairs;
  const int blk = blockIdx.x - G.blk_half;
  const int lane_ = threadIdx.x & 63;
  const int gl = blk * 64 + lane_;
  const int nlanes = npairs * NB;
  const int g = gl < nlanes ? gl : nlanes - 1;
  const int pair = g / NB;
  const int d_ = g % NB;
  const size_t base = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K_, NB);
  const s4 *sp0_ = SP0 + base;
  s2 *xp1_ = XP1 + base;
  const s2 *p1_ = XP1 + plane + base;
  s2 *A_ = Aarr + base;
  uint32_t *D_ = Darr + G.dw0 + (size_t)pair * dec_words(K_, NB);
  const s2 *tl_ = T + (size_t)(G.pair0 + pair) * 12;
  const int pe = t4_pair_elems(K_, NB), pw = (blk * 64) / NB;
  const size_t wb = (size_t)G.elem0 + (size_t)pw * pe;
  const s4 *wsp0_ = SP0 + wb;
  s2 *wx2_ = XP1 + wb, *wa_ = Aarr + wb;
  const s2 *wp1_ = XP1 + plane + wb;
  const uint32_t po_ = (uint32_t)((pair - pw) * pe) * 4u;
  const uint16_t *fwd0 = G.fwd, *rev0 = G.rev;
  for (int n = n0; n < n0 + nh; n++) {
    const bool dec = dout && n + 1 == n0 + nh;
    if (n > n0) __syncthreads(); // the previous half-iteration's stores and LDS reads are done
    // opaque copies of the loop invariants: without them the compiler hoists every body's
    // address arithmetic out of the half-iteration loop, and the five bodies' hoisted values
    // together no longer fit the register file (scratch spills)
    // The copies go through the asm as global (address space 1) pointers: a generic pointer that
    // leaves an asm is of unknown space to the compiler, and every access through it would be a
    // flat instruction, which counts against lgkmcnt too (the checkpoint LDS waits would then wait
    // for the chunk prefetches). The casts back to generic are address-space casts from global,
    // which the address-space inference folds into global loads and stores.
    gptr_t<s4> gsp0 = gptr(sp0_);
    gmut_t<s2> gxp1 = gmut<s2>(xp1_), gA = gmut<s2>(A_);
    gptr_t<s2> gp1 = gptr(p1_), gtl = gptr(tl_);
    gmut_t<uint32_t> gD = gmut<uint32_t>(D_);
    gptr_t<uint16_t> fwd = gptr(fwd0), rev = gptr(rev0);
    int K = K_, d = d_, lane = lane_;
    uint32_t po = po_;
    gptr_t<s4> wsp0 = gptr(wsp0_);
    gptr_t<s2> wp1 = gptr(wp1_);
    gmut_t<s2> wx2 = gmut<s2>(wx2_), wa = gmut<s2>(wa_);
    asm volatile("" : "+v"(gsp0), "+v"(gxp1), "+v"(gA), "+v"(gp1), "+v"(gtl), "+v"(gD), "+v"(d), "+v"(lane), "+v"(po));
    asm volatile("" : "+s"(fwd), "+s"(rev), "+s"(K), "+s"(wsp0), "+s"(wp1), "+s"(wx2), "+s"(wa));
    WinRes R;
    R.sp0 = mk_rsrc((const void *)wsp0);
    R.x2 = mk_rsrc((const void *)wx2);
    R.p1 = mk_rsrc((const void *)wp1);
    R.a = mk_rsrc((const void *)wa);
    R.tb = mk_rsrc((const void *)((n & 1) ? fwd : rev));
    R.po = po;
    const s4 *sp0 = (const s4 *)gsp0;
    s2 *xp1 = (s2 *)gxp1, *A = (s2 *)gA;
    const s2 *p1 = (const s2 *)gp1, *tl = (const s2 *)gtl;
    uint32_t *D = (uint32_t *)gD;
    if (n & 1) {
      if (dec)
        win_bidir_body<NB, DIV, 1, true, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
      else
        win_bidir_body<NB, DIV, 1, false, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
    } else if (n == 0) {
      win_bidir_body<NB, DIV, 2, false, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
    } else {
      if (dec)
        win_bidir_body<NB, DIV, 0, true, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
      else
        win_bidir_body<NB, DIV, 0, false, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
    }
  }
}

// After half-iteration n of the workgroup's pairs (their decision words in D, written by this
// workgroup before the barrier): the CRC of every unfinished code block, as k_decide folds it
// (crc.c:144-155 is linear: XOR of the chain-major weights TdGroup::wc over the set decision
// bits), the done / ok / noi update of sch.c:361-391, and the natural-order bytes of the blocks
// that end at this half-iteration (via Dfz / cb_end and k_es_bytes). Returns (uniformly) whether
// every block of the workgroup is done.
template <int NB>
__device__ __noinline__ bool es_check(const TdGroup &G, const int *wpair, int n, const uint32_t *__restrict__ Darr,
                                      const TdEs &es, uint32_t *red, int *fin) {
  constexpr int NP = 64 / NB; // pairs per workgroup (wpair[lp]: their group-local pair numbers)
  const int K = G.K;
  const int L = K / NB, G16 = (L + 15) / 16, nw = NB * G16;
  const bool dec2 = n & 1;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const gptr_t<uint32_t> wc = gptr(G.wc[dec2 ? 1 : 0]);
  // per pair: done flags after the previous half-iteration (fin bit 0; finished blocks are skipped)
  bool skip[NP][2];
#pragma unroll
  for (int lp = 0; lp < NP; lp++) {
    skip[lp][0] = fin[2 * lp] & 1;
    skip[lp][1] = fin[2 * lp + 1] & 1;
  }
#pragma unroll
  for (int lp = 0; lp < NP; lp++) {
    uint32_t c0 = 0, c1 = 0;
    if (!(skip[lp][0] && skip[lp][1])) {
      const gptr_t<uint32_t> dw = gptr(Darr + G.dw0 + (size_t)wpair[lp] * nw);
      for (int q = t; q < nw; q += 128) {
        const uint32_t w = dw[q];
        if (w == 0u) continue;
        const gptr_t<u4> wq = (gptr_t<u4>)(wc + (size_t)q * 16);
        uint32_t wt[16];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const u4 v = wq[i];
          wt[4 * i] = v[0];
          wt[4 * i + 1] = v[1];
          wt[4 * i + 2] = v[2];
          wt[4 * i + 3] = v[3];
        }
#pragma unroll
        for (int j = 0; j < 16; j++) {
          c0 ^= ((w >> j) & 1u) ? wt[j] : 0u;
          c1 ^= ((w >> (16 + j)) & 1u) ? wt[j] : 0u;
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      c0 ^= __shfl_xor(c0, o);
      c1 ^= __shfl_xor(c1, o);
    }
    if (lane == 0) {
      red[(lp * 2 + 0) * 2 + wv] = c0;
      red[(lp * 2 + 1) * 2 + wv] = c1;
    }
  }
  __syncthreads();
  if (t < 2 * NP) {
    const int lp = t >> 1, h = t & 1;
    int done = 1, now = 0;
    if (!skip[lp][h]) {
      const int cb = G.cb0 + 2 * wpair[lp] + h;
      const uint32_t crc = red[t * 2] ^ red[t * 2 + 1];
      es.noi[cb] = (uint32_t)(n + 1);
      if (crc == 0u) {
        es.cb_ok[cb] = 1;
        es.cb_done[cb] = 1;
        now = 1;
      } else if (n + 1 >= es.max_halfits) {
        es.cb_done[cb] = 1;
        now = 1;
      } else {
        done = 0;
      }
    }
    fin[t] = done | (now << 1);
  }
  __syncthreads();
  // The blocks that ended now keep their decision words: copied (their 16-bit halves) into the
  // frozen plane Dfz, the half-iteration's parity in cb_end; k_es_bytes turns them into bytes
  // after the launches (a byte loop here held the workgroup, and with it its CU's LDS, for
  // ~100 us per launch).
  bool all = true;
#pragma unroll
  for (int lp = 0; lp < NP; lp++) {
    const int f0 = fin[lp * 2], f1 = fin[lp * 2 + 1];
    all = all && (f0 & 1) && (f1 & 1);
    const uint32_t mask = ((f0 & 2) ? 0xffffu : 0u) | ((f1 & 2) ? 0xffff0000u : 0u);
    if (!mask) continue;
    const gptr_t<uint32_t> dw = gptr(Darr + G.dw0 + (size_t)wpair[lp] * nw);
    const gmut_t<uint32_t> fz = gmut<uint32_t>(es.dfz + G.dw0 + (size_t)wpair[lp] * nw);
    for (int q = t; q < nw; q += 128) fz[q] = (fz[q] & ~mask) | (dw[q] & mask);
    if (t < 2 && (fin[lp * 2 + t] & 2)) es.cb_end[G.cb0 + 2 * wpair[lp] + t] = (uint8_t)(1 + (n & 1));
  }
  return all;
}

// The early-stop form of k_win_bidir_run (the DL-SCH path: srslte_tdec_iteration + CRC check per
// half-iteration, sch.c:361-391): up to max_halfits half-iterations in ONE launch; after each one
// the workgroup checks the CRC of its own code blocks (es_check) and leaves once all of them are
// done, so a batch at high SNR costs the half-iterations its blocks need and no decide launches.
// Blocks done at entry (HARQ retransmissions whose CRC passed before, cb_done seeded) are
// skipped; a partly finished workgroup decodes on, its finished blocks' results stay frozen.
// es.prio raises its waves' issue priority (wave_prio.h): it runs a few workgroups beside other
// streams' throughput kernels.
template <int NB, int DIV, bool B8>
__global__ __launch_bounds__(128, TD_BIDIR_WAVES) void k_win_bidir_es(const TdGroup *__restrict__ groups, int ngroups,
                                                      const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                      s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                      const s2 *__restrict__ T, size_t plane, TdEs es) {
  extern __shared__ s4 cks[];
  constexpr int NP = 64 / NB; // pairs per workgroup
  __shared__ uint32_t red[NP * 2 * 2];
  __shared__ int fin[NP * 2];
  __shared__ int wpair[NP];
  wave_prio(es.prio);
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int K_ = G.K, npairs = G.npairs;
  const int blk = blockIdx.x - G.blk_half;
  // The workgroup's pairs: NP consecutive ones, or with es.run_list (the hybrid schedule, after the
  // first half-iteration's k_decide) entries NP blk .. of the group's list of pairs still running
  // (run_cnt[pair0] of them): the few stragglers are packed into few workgroups, and the rest of the
  // launch's workgroups leave at once instead of holding a CU's SIMDs each for one running block.
  // A list slot past the count repeats the workgroup's first pair, marked done (never checked).
  const int nrun = es.run_list ? (int)es.run_cnt[G.pair0] : 0;
  if (es.run_list && NP * blk >= nrun) return;
  if (threadIdx.x < NP) {
    const int lp = threadIdx.x;
    int p;
    if (es.run_list) {
      const int j = NP * blk + lp;
      p = (int)es.run_list[G.pair0 + (j < nrun ? j : NP * blk)];
      if (j >= nrun) p = -1 - p;
    } else {
      p = NP * blk + lp;
      if (p >= npairs) p = -1 - (npairs - 1);
    }
    wpair[lp] = p;
  }
  __syncthreads();
  // fin[2 lp + h]: bit 0 = CB h of the workgroup's pair lp is done (seeded from cb_done: HARQ
  // blocks that passed earlier; absent blocks count as done), bit 1 = it ended at this check
  if (threadIdx.x < 2 * NP) {
    const int p = wpair[threadIdx.x >> 1], h = threadIdx.x & 1;
    fin[threadIdx.x] = (p < 0 || 2 * p + h >= G.ncb || es.cb_done[G.cb0 + 2 * p + h]) ? 1 : 0;
  }
  __syncthreads();
  {
    bool all_done = true;
    for (int i = 0; i < 2 * NP; i++) all_done = all_done && (fin[i] & 1);
    if (all_done) return;
  }
  if (threadIdx.x < NP && wpair[threadIdx.x] < 0) wpair[threadIdx.x] = -1 - wpair[threadIdx.x]; // a real pair
  __syncthreads();
  const int lane_ = threadIdx.x & 63;
  const int pair = wpair[lane_ / NB]; // lanes of a repeated slot redo that pair: same values, same addresses
  const int d_ = lane_ % NB;
  const size_t base = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K_, NB);
  const s4 *sp0_ = SP0 + base;
  s2 *xp1_ = XP1 + base;
  const s2 *p1_ = XP1 + plane + base;
  s2 *A_ = Aarr + base;
  uint32_t *D_ = Darr + G.dw0 + (size_t)pair * dec_words(K_, NB);
  const s2 *tl_ = T + (size_t)(G.pair0 + pair) * 12;
  // wave bases at the group's first pair, each lane's pair by its offset (any pair of the group)
  const int pe = t4_pair_elems(K_, NB), pw = 0;
  const size_t wb = (size_t)G.elem0 + (size_t)pw * pe;
  const s4 *wsp0_ = SP0 + wb;
  s2 *wx2_ = XP1 + wb, *wa_ = Aarr + wb;
  const s2 *wp1_ = XP1 + plane + wb;
  const uint32_t po_ = (uint32_t)((pair - pw) * pe) * 4u;
  const uint16_t *fwd0 = G.fwd, *rev0 = G.rev;
  for (int n = es.n0; n < es.n1; n++) {
    if (n > es.n0) __syncthreads();
    // opaque loop-invariant copies, global address space (see k_win_bidir_run)
    gptr_t<s4> gsp0 = gptr(sp0_);
    gmut_t<s2> gxp1 = gmut<s2>(xp1_), gA = gmut<s2>(A_);
    gptr_t<s2> gp1 = gptr(p1_), gtl = gptr(tl_);
    gmut_t<uint32_t> gD = gmut<uint32_t>(D_);
    gptr_t<uint16_t> fwd = gptr(fwd0), rev = gptr(rev0);
    int K = K_, d = d_, lane = lane_;
    uint32_t po = po_;
    gptr_t<s4> wsp0 = gptr(wsp0_);
    gptr_t<s2> wp1 = gptr(wp1_);
    gmut_t<s2> wx2 = gmut<s2>(wx2_), wa = gmut<s2>(wa_);
    asm volatile("" : "+v"(gsp0), "+v"(gxp1), "+v"(gA), "+v"(gp1), "+v"(gtl), "+v"(gD), "+v"(d), "+v"(lane), "+v"(po));
    asm volatile("" : "+s"(fwd), "+s"(rev), "+s"(K), "+s"(wsp0), "+s"(wp1), "+s"(wx2), "+s"(wa));
    WinRes R;
    R.sp0 = mk_rsrc((const void *)wsp0);
    R.x2 = mk_rsrc((const void *)wx2);
    R.p1 = mk_rsrc((const void *)wp1);
    R.a = mk_rsrc((const void *)wa);
    R.tb = mk_rsrc((const void *)((n & 1) ? fwd : rev));
    R.po = po;
    const s4 *sp0 = (const s4 *)gsp0;
    s2 *xp1 = (s2 *)gxp1, *A = (s2 *)gA;
    const s2 *p1 = (const s2 *)gp1, *tl = (const s2 *)gtl;
    uint32_t *D = (uint32_t *)gD;
    if (n & 1)
      win_bidir_body<NB, DIV, 1, true, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
    else if (n == 0)
      win_bidir_body<NB, DIV, 2, true, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
    else
      win_bidir_body<NB, DIV, 0, true, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
    __syncthreads(); // the half-iteration's decision words of both waves are written
    if (es_check<NB>(G, wpair, n, Darr, es, red, fin)) break;
  }
}

// ------------------------------------------------------------------ first half-iteration + check ----
// The hybrid schedule's first half-iteration (DEC1, n = 0) with the decide of its own blocks fused in
// (TdEs::bytes_direct, SRSGPU_H0_DECIDE): k_win_bidir's body, then the workgroup stages its pairs'
// decision words in the checkpoint LDS (free after the body) and does what k_decide does for them —
// the CRC of each block (the chain-major weights TdGroup::wc, crc.c:144-155 is linear), done / ok /
// noi (sch.c:361-391), the natural-order bytes of the blocks that pass (turbodecoder.c:353-360 +
// decision_byte, MSB first), and the pairs still running appended to their group's list for the
// early-stop launch (TdEs::list_out / cnt_out).
// Bytes from the staged words: natural position p = d L + k is step k of chain d, bit (c & 15) + 16 h
// of word c >> 4 with c = p + d (16 G16 - L); the threads take 32-bit output words, a byte inside one
// chain is 8 consecutive bits of it (two 16-bit halves funnelled), a byte across a chain boundary
// goes bit by bit.
__device__ __forceinline__ uint32_t h0_byte(const uint32_t *dw, int nw, int L, int gap, float invL, int h, int p) {
  const int d = (int)(((float)p + 0.5f) * invL); // exact: see k_decide
  const int k0 = p - d * L;
  uint32_t v;
  if (k0 + 7 < L) {
    const int c = p + d * gap, q = c >> 4;
    const uint32_t lo = (dw[q] >> (16 * h)) & 0xffffu;
    const uint32_t hi = q + 1 < nw ? (dw[q + 1] >> (16 * h)) & 0xffffu : 0u;
    v = ((lo | (hi << 16)) >> (c & 15)) & 0xffu;
  } else {
    v = 0;
    for (int i = 0; i < 8; i++) {
      const int pi = p + i;
      const int di = (int)(((float)pi + 0.5f) * invL);
      const int c = pi + di * gap;
      v |= ((dw[c >> 4] >> ((c & 15) + 16 * h)) & 1u) << i;
    }
  }
  return __builtin_bitreverse32(v) >> 24;
}

template <int NB>
__device__ __noinline__ void h0_check(const TdGroup &G, const int *wpair, const uint32_t *__restrict__ Darr,
                                      const TdEs &es, uint32_t *red, int *fin, uint32_t *sdw) {
  constexpr int NP = 64 / NB;
  const int K = G.K, L = K / NB, G16 = (L + 15) / 16, nw = NB * G16, gap = 16 * G16 - L;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // the pairs' decision words into LDS (coalesced, all loads up front)
  for (int i = t; i < NP * nw; i += 128) {
    const int lp = i / nw, q = i - lp * nw;
    sdw[i] = Darr[G.dw0 + (size_t)wpair[lp] * nw + q];
  }
  __syncthreads();
  const gptr_t<uint32_t> wc = gptr(G.wc[0]);
#pragma unroll
  for (int lp = 0; lp < NP; lp++) {
    uint32_t c0 = 0, c1 = 0;
    if (!((fin[2 * lp] & 1) && (fin[2 * lp + 1] & 1))) {
      for (int q = t; q < nw; q += 128) {
        const uint32_t w = sdw[lp * nw + q];
        if (w == 0u) continue;
        const gptr_t<u4> wq = (gptr_t<u4>)(wc + (size_t)q * 16);
        uint32_t wt[16];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const u4 v = wq[i];
          wt[4 * i] = v[0];
          wt[4 * i + 1] = v[1];
          wt[4 * i + 2] = v[2];
          wt[4 * i + 3] = v[3];
        }
#pragma unroll
        for (int j = 0; j < 16; j++) {
          c0 ^= ((w >> j) & 1u) ? wt[j] : 0u;
          c1 ^= ((w >> (16 + j)) & 1u) ? wt[j] : 0u;
        }
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      c0 ^= __shfl_xor(c0, o);
      c1 ^= __shfl_xor(c1, o);
    }
    if (lane == 0) {
      red[(lp * 2 + 0) * 2 + wv] = c0;
      red[(lp * 2 + 1) * 2 + wv] = c1;
    }
  }
  __syncthreads();
  if (t < 2 * NP) {
    const int lp = t >> 1, h = t & 1;
    int done = 1, now = 0;
    if (!(fin[t] & 1)) {
      const int cb = G.cb0 + 2 * wpair[lp] + h;
      const uint32_t crc = red[t * 2] ^ red[t * 2 + 1];
      es.noi[cb] = 1u;
      if (crc == 0u) {
        es.cb_ok[cb] = 1;
        es.cb_done[cb] = 1;
        now = 1;
      } else if (1 >= es.max_halfits) {
        es.cb_done[cb] = 1;
        now = 1;
      } else {
        done = 0;
      }
    }
    fin[t] = done | (now << 1);
  }
  __syncthreads();
  if (es.list_out && t < NP && !((fin[2 * t] & 1) && (fin[2 * t + 1] & 1)))
    es.list_out[G.pair0 + atomicAdd(&es.cnt_out[G.pair0], 1u)] = (uint32_t)wpair[t];
  // bytes of the blocks that ended now, 32-bit words (rows are 4-byte aligned when outb and the
  // stride are; otherwise bytes)
  const float invL = 1.0f / (float)L;
  const int nbytes = K / 8, nwd = nbytes / 4;
  const bool w32 = ((uintptr_t)es.outb & 3u) == 0 && (es.out_stride & 3u) == 0;
#pragma unroll
  for (int lp = 0; lp < NP; lp++) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      if (!(fin[2 * lp + h] & 2)) continue;
      const uint32_t *dw = sdw + lp * nw;
      uint8_t *row = es.outb + (size_t)(G.cb0 + 2 * wpair[lp] + h) * es.out_stride;
      if (w32) {
        for (int w = t; w < nwd; w += 128) {
          const int p = 32 * w;
          gmut<uint32_t>(row)[w] = h0_byte(dw, nw, L, gap, invL, h, p) | (h0_byte(dw, nw, L, gap, invL, h, p + 8) << 8) |
                                   (h0_byte(dw, nw, L, gap, invL, h, p + 16) << 16) |
                                   (h0_byte(dw, nw, L, gap, invL, h, p + 24) << 24);
        }
        for (int b = 4 * nwd + t; b < nbytes; b += 128) gmut<uint8_t>(row)[b] = (uint8_t)h0_byte(dw, nw, L, gap, invL, h, 8 * b);
      } else {
        for (int b = t; b < nbytes; b += 128) gmut<uint8_t>(row)[b] = (uint8_t)h0_byte(dw, nw, L, gap, invL, h, 8 * b);
      }
    }
  }
}

template <int NB, int DIV, bool B8>
__global__ __launch_bounds__(128, TD_BIDIR_WAVES) void k_win_bidir_h0c(const TdGroup *__restrict__ groups, int ngroups,
                                                       const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                       s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                       const s2 *__restrict__ T, size_t plane, TdEs es) {
  extern __shared__ s4 cks[];
  constexpr int NP = 64 / NB;
  __shared__ uint32_t red[NP * 2 * 2];
  __shared__ int fin[NP * 2];
  __shared__ int wpair[NP];
  wave_prio(es.prio);
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); // 0: alpha, 1: beta
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int K = G.K, npairs = G.npairs;
  const int blk = blockIdx.x - G.blk_half;
  const int lane = threadIdx.x & 63;
  // k_win_bidir's mapping: NP consecutive pairs, lanes past the group's chains repeat its last pair
  // (their slots count as done: never checked, never listed)
  if (threadIdx.x < 2 * NP) {
    const int p = NP * blk + (threadIdx.x >> 1), h = threadIdx.x & 1;
    fin[threadIdx.x] = (p >= npairs || 2 * p + h >= G.ncb || es.cb_done[G.cb0 + 2 * p + h]) ? 1 : 0;
    if (h == 0) wpair[threadIdx.x >> 1] = p < npairs ? p : npairs - 1;
  }
  __syncthreads();
  {
    bool all_done = true;
    for (int i = 0; i < 2 * NP; i++) all_done = all_done && (fin[i] & 1);
    if (all_done) return; // HARQ blocks that passed before: both waves leave before the barriers
  }
  const int gl = blk * 64 + lane;
  const int nlanes = npairs * NB;
  const int g = gl < nlanes ? gl : nlanes - 1;
  const int pair = g / NB;
  const int d = g % NB;
  const size_t base = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, NB);
  const s4 *sp0 = SP0 + base;
  s2 *xp1 = XP1 + base;
  const s2 *p1 = XP1 + plane + base;
  s2 *A = Aarr + base;
  uint32_t *D = Darr + G.dw0 + (size_t)pair * dec_words(K, NB);
  const s2 *tl = T + (size_t)(G.pair0 + pair) * 12;
  const WinRes R = win_res<NB>(G, K, blk, pair, SP0, XP1, Aarr, plane, G.rev);
  win_bidir_body<NB, DIV, 2, true, B8>(sp0, xp1, p1, A, D, tl, R, cks, K, d, role, lane);
  __syncthreads(); // both waves' decision words are written; the checkpoint LDS is free
  h0_check<NB>(G, wpair, Darr, es, red, fin, reinterpret_cast<uint32_t *>(cks));
}

// ------------------------------------------------------------------ SSE non-window ----
#define TD_SP 8 // steps per prefetch group of the sequential decoders: must divide 8 (every LTE K is a multiple of 8, not of 16)
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
  const size_t base = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, 1);
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
  // every LTE K is a multiple of 8: the recursion runs in groups of TD_SP steps whose inputs were
  // loaded one group ahead (the loads do not depend on the recursion; one serial chain per lane
  // leaves nothing else to hide their latency)
  constexpr int P = TD_SP;
  StepIn nx[P];
#pragma unroll
  for (int u = 0; u < P; u++) nx[u] = load_step<MODE, true>(sp0, xp1, p1, A, u);
  for (int k0 = 0; k0 < K; k0 += P) { // :211-297
    StepIn cu[P];
#pragma unroll
    for (int u = 0; u < P; u++) cu[u] = nx[u];
    const int kn = min(k0 + P, K - P);
#pragma unroll
    for (int u = 0; u < P; u++) nx[u] = load_step<MODE, true>(sp0, xp1, p1, A, kn + u);
#pragma unroll
    for (int u = 0; u < P; u++) {
      const int k = k0 + u;
      const StepIn &s = cu[u];
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
  }
  s2 b[8];
  b[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) b[i] = splat(-TD_INF);
  uint32_t dacc = 0;
  // :105-206. Tail steps K+2 .. K (no LLR), then steps K-1 .. 0 in groups of TD_SP whose inputs,
  // stored alphas and scatter targets were loaded one group ahead.
  auto bsteps = [&](s2 g0, s2 g1, s2 bp[8], s2 bn[8]) {
    bp[0] = wadd(b[4], g1); bp[1] = wadd(b[0], g1); bp[2] = wadd(b[1], g0); bp[3] = wadd(b[5], g0);
    bp[4] = wadd(b[6], g0); bp[5] = wadd(b[2], g0); bp[6] = wadd(b[3], g1); bp[7] = wadd(b[7], g1);
    bn[0] = wsub(b[0], g1); bn[1] = wsub(b[4], g1); bn[2] = wsub(b[5], g0); bn[3] = wsub(b[1], g0);
    bn[4] = wsub(b[2], g0); bn[5] = wsub(b[6], g0); bn[6] = wsub(b[7], g1); bn[7] = wsub(b[3], g1);
#pragma unroll
    for (int i = 0; i < 8; i++) b[i] = smax(bp[i], bn[i]);
  };
  for (int k = K + 2; k >= K; k--) {
    const s2 x = tl[tail_xoff + 2 * (k - K)], y = tl[tail_xoff + 2 * (k - K) + 1];
    const s2 g0 = s2{(short)(((int)x.x - y.x) / 2), (short)(((int)x.y - y.y) / 2)};
    const s2 g1 = s2{(short)(((int)x.x + y.x) / 2), (short)(((int)x.y + y.y) / 2)};
    s2 bp[8], bn[8];
    bsteps(g0, g1, bp, bn);
  }
  StepIn ns[P];
  s2 na[P][8];
  int nt[P];
  auto fetch = [&](int k1, StepIn *fs, s2 (*fa)[8], int *ft) {
#pragma unroll
    for (int u = 0; u < P; u++) {
      const int k = k1 - u;
      fs[u] = load_step<MODE, true>(sp0, xp1, p1, A, k);
#pragma unroll
      for (int i = 0; i < 8; i++) fa[u][i] = AL(k, i);
      ft[u] = tbl[k];
    }
  };
  fetch(K - 1, ns, na, nt);
  for (int k1 = K - 1; k1 >= 0; k1 -= P) {
    StepIn cs[P];
    s2 ca[P][8];
    int ct[P];
#pragma unroll
    for (int u = 0; u < P; u++) {
      cs[u] = ns[u];
      ct[u] = nt[u];
#pragma unroll
      for (int i = 0; i < 8; i++) ca[u][i] = na[u][i];
    }
    fetch(max(k1 - P, P - 1), ns, na, nt);
#pragma unroll
    for (int u = 0; u < P; u++) {
      const int k = k1 - u;
      const StepIn &st = cs[u];
      const s2 g1 = wadd(st.x, st.y) >> 1, g0 = wsub(st.x, st.y) >> 1;
      s2 bp[8], bn[8];
      bsteps(g0, g1, bp, bn);
      s2 mp = splat(-32768), mn = splat(-32768);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        mp = smax(mp, wadd(bp[i], ca[u][i]));
        mn = smax(mn, wadd(bn[i], ca[u][i]));
      }
      // hMax(bn) - hMax(bp) with hMax(v) = 0x7FFF - max(v) (minpos_epu16 trick, :97-102)
      const s2 llr = wsub(wsub(splat(0x7FFF), mn), wsub(splat(0x7FFF), mp));
      store_out<MODE == 1>(xp1, A, ct[u], llr, st.e);
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

// The SSE decoder run bidirectionally: the same arithmetic as k_sse_halfit, half its serial
// chain. Two waves per 64 CB pairs, wave 0 owns the alpha recursion, wave 1 the beta recursion.
//   phase 1  wave 0: alphas of steps 0..M-1, stored as k_sse_halfit stores them (AL(k) = the
//            state leaving step k-1, before its normalisation); wave 1: the tail steps, then the
//            betas of steps K-1..M, storing B(k) = the state entering step k in the scratch slot
//            AL(k), k >= M (no alpha past M is stored, so the slots are free).
//   phase 2  (after one workgroup barrier) wave 0 runs the alphas of steps M..K-1 and emits their
//            LLRs from its own AL(k) and the stored B(k); wave 1 runs the betas of steps M-1..0 and
//            emits their LLRs from its own B(k) and the stored AL(k).
// Each recursion keeps the reference's order and normalisation steps and every LLR combines the
// same AL(k), B(k) and branch metrics as turbodecoder_sse.c:105-206, so the outputs are
// bit-identical to k_sse_halfit. M = 16*floor(K/32) is a multiple of 16, so the two waves'
// decision words never share a word.
// Buffer addressing of the SSE decoders: per-group resources (SGPRs), per-lane byte offsets fixed
// for the launch (VGPRs) and per-step offsets that are wave-uniform (SGPRs), so no load or store
// needs per-access VGPR address arithmetic (the flat 64-bit form spent one v_lshl_add_u64 and an
// s_add/s_addc pair per access, more than the recursions themselves).
struct SseRes {
  rsrc_t sp0, x2, p1, a, sc, d;
  uint32_t vo8, vo4, vsc, vd; // lane offsets: SP0 (8-byte elements), X2/P1/A, scratch, D
  uint32_t row;               // bytes per scratch row (one state of one step for every pair)
};
__device__ __forceinline__ void bst32s(uint32_t v, rsrc_t r, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, vo, so, 0);
}
__device__ __forceinline__ s2 u2s(uint32_t v) { return __builtin_bit_cast(s2, v); }
__device__ __forceinline__ uint32_t s2u(s2 v) { return __builtin_bit_cast(uint32_t, v); }
// the inputs of step k as load_step<MODE, true> reads them (SSE: wrapping app add)
template <int MODE>
__device__ __forceinline__ StepIn sse_ld(const SseRes &R, int k) {
  StepIn r;
  if (MODE == 1) {
    r.x = u2s(bld32(R.x2, R.vo4, (uint32_t)k * 4));
    r.y = u2s(bld32(R.p1, R.vo4, (uint32_t)k * 4));
    r.e = r.x;
  } else {
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    const u2v v = __builtin_bit_cast(u2v, __builtin_amdgcn_raw_buffer_load_b64(R.sp0, R.vo8, (uint32_t)k * 8, 0));
    const s2 a = MODE == 2 ? splat(0) : u2s(bld32(R.a, R.vo4, (uint32_t)k * 4));
    r.x = wadd(u2s(v.x), a);
    r.y = u2s(v.y);
    r.e = a;
  }
  return r;
}

// One half-iteration of the workgroup's 64 pairs; pair p = this lane's pair within the group;
// `done` lanes (finished pairs, lanes past the group) touch no memory but reach the barrier.
template <int MODE>
__device__ __forceinline__ void sse_bidir_body(const TdGroup &G, int p, bool done,
                                               const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                               s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                               const s2 *__restrict__ T, size_t plane,
                                               s2 *__restrict__ scratch_base) {
  const int K = G.K, npairs = G.npairs;
  const int role = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); // 0: alpha, 1: beta
  const int pair = p < npairs ? p : npairs - 1;
  const uint32_t pe = (uint32_t)t4_pair_elems(K, 1);
  SseRes R;
  R.sp0 = mk_rsrc(SP0 + G.elem0);
  R.x2 = mk_rsrc(XP1 + G.elem0);
  R.p1 = mk_rsrc(XP1 + plane + G.elem0);
  R.a = mk_rsrc(Aarr + G.elem0);
  R.sc = mk_rsrc(scratch_base + G.sc0);
  R.d = mk_rsrc(Darr ? Darr + G.dw0 : Darr);
  R.vo8 = (uint32_t)pair * pe * 8;
  R.vo4 = (uint32_t)pair * pe * 4;
  R.vsc = (uint32_t)pair * 4;
  R.vd = (uint32_t)pair * (uint32_t)dec_words(K, 1) * 4;
  R.row = (uint32_t)npairs * 4;
  const bool dout = Darr != nullptr;
  const s2 *tl = T + (size_t)(G.pair0 + pair) * 12;
  // the scatter table of the half-iteration, 8 entries (one aligned 16-byte word) per step group,
  // read through the constant address space: a scalar load into SGPRs (wave-uniform targets, used
  // as buffer soffsets), waited on with lgkmcnt rather than behind the vector prefetches
  typedef const __attribute__((address_space(4))) u4 cu4;
  cu4 *tb4 = (cu4 *)(const __attribute__((address_space(4))) void *)(uintptr_t)(MODE == 1 ? G.fwd : G.rev);
  auto tbl8 = [&](int k0, int *t) { // k0 a multiple of 8: entries k0 .. k0 + 7
    const u4 w = tb4[k0 >> 3];
#pragma unroll
    for (int u = 0; u < 8; u++) t[u] = (int)((w[u >> 1] >> (16 * (u & 1))) & 0xffffu);
  };
  auto al_ld = [&](int k, int i) { return u2s(bld32(R.sc, R.vsc, ((uint32_t)k * 8 + i) * R.row)); };
  auto al_st = [&](int k, int i, s2 v) { bst32s(s2u(v), R.sc, R.vsc, ((uint32_t)k * 8 + i) * R.row); };
  auto out_st = [&](int t, s2 llr, s2 e) { // store_out: DEC1 E' into app2, DEC2 into A
    bst32s(s2u(wsub(llr, e)), MODE == 1 ? R.a : R.x2, R.vo4, (uint32_t)t * 4);
  };
  const int M = 16 * (K / 32); // K >= 40, a multiple of 8: 16 <= M <= K/2
  constexpr int P = TD_SP;
  static_assert(P == 8, "tbl8 loads 8 scatter targets per step group");
  // beta candidates of one step (bp: bit 1, bn: bit 0) and the LLR against the alphas aa
  auto bpn = [](const s2 bb[8], s2 g0, s2 g1, s2 bp[8], s2 bn[8]) {
    bp[0] = wadd(bb[4], g1); bp[1] = wadd(bb[0], g1); bp[2] = wadd(bb[1], g0); bp[3] = wadd(bb[5], g0);
    bp[4] = wadd(bb[6], g0); bp[5] = wadd(bb[2], g0); bp[6] = wadd(bb[3], g1); bp[7] = wadd(bb[7], g1);
    bn[0] = wsub(bb[0], g1); bn[1] = wsub(bb[4], g1); bn[2] = wsub(bb[5], g0); bn[3] = wsub(bb[1], g0);
    bn[4] = wsub(bb[2], g0); bn[5] = wsub(bb[6], g0); bn[6] = wsub(bb[7], g1); bn[7] = wsub(bb[3], g1);
  };
  auto llr_of = [](const s2 bp[8], const s2 bn[8], const s2 aa[8]) -> s2 {
    s2 mp = splat(-32768), mn = splat(-32768);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      mp = smax(mp, wadd(bp[i], aa[i]));
      mn = smax(mn, wadd(bn[i], aa[i]));
    }
    return wsub(wsub(splat(0x7FFF), mn), wsub(splat(0x7FFF), mp)); // hMax(bn) - hMax(bp)
  };
  auto astep = [](const s2 a[8], s2 g0, s2 g1, s2 n[8]) { // :211-297
    n[0] = smax(wadd(a[1], g1), wsub(a[0], g1));
    n[1] = smax(wadd(a[2], g0), wsub(a[3], g0));
    n[2] = smax(wadd(a[5], g0), wsub(a[4], g0));
    n[3] = smax(wadd(a[6], g1), wsub(a[7], g1));
    n[4] = smax(wadd(a[0], g1), wsub(a[1], g1));
    n[5] = smax(wadd(a[3], g0), wsub(a[2], g0));
    n[6] = smax(wadd(a[4], g0), wsub(a[5], g0));
    n[7] = smax(wadd(a[7], g1), wsub(a[6], g1));
  };
  auto norm = [](s2 v[8]) {
    const s2 z = v[0];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = wsub(v[i], z);
  };
  uint32_t dacc = 0;
  if (role == 0) {
    s2 a[8], apre[8]; // a: the recursion state, apre: AL(k) of the next step
    a[0] = splat(0);
#pragma unroll
    for (int i = 1; i < 8; i++) a[i] = splat(-TD_INF);
#pragma unroll
    for (int i = 0; i < 8; i++) apre[i] = a[i];
    if (!done) { // phase 1: alphas of steps 0..M-1 (groups of 8: k & 3 known per unrolled step)
#pragma unroll
      for (int i = 0; i < 8; i++) al_st(0, i, a[i]);
      StepIn nx[P];
#pragma unroll
      for (int u = 0; u < P; u++) nx[u] = sse_ld<MODE>(R, u);
      for (int g = 0; g < M / P; g++) {
        const int k0 = g * P;
        StepIn cu[P];
#pragma unroll
        for (int u = 0; u < P; u++) cu[u] = nx[u];
#pragma unroll
        for (int u = 0; u < P; u++) nx[u] = sse_ld<MODE>(R, k0 + P + u); // < K: M <= K - 8
#pragma unroll
        for (int u = 0; u < P; u++) {
          const s2 g1 = wadd(cu[u].x, cu[u].y) >> 1, g0 = wsub(cu[u].x, cu[u].y) >> 1;
          s2 n[8];
          astep(a, g0, g1, n);
#pragma unroll
          for (int i = 0; i < 8; i++) {
            a[i] = n[i];
            apre[i] = n[i];
          }
          if (u < P - 1 || k0 + P < M) { // AL(M) is the beta wave's slot
#pragma unroll
            for (int i = 0; i < 8; i++) al_st(k0 + u + 1, i, n[i]);
          }
          if ((u & 3) == 3) norm(a);
        }
      }
    }
    __syncthreads();
    if (done) return;
    // phase 2: alphas and LLRs of steps M..K-1; inputs, stored betas and scatter targets are
    // loaded one group ahead
    StepIn nx[P];
    s2 nb[P][8];
    int nt[P];
    auto fetch = [&](int k1, StepIn *fs, s2 (*fb)[8], int *ft) {
#pragma unroll
      for (int u = 0; u < P; u++) {
        fs[u] = sse_ld<MODE>(R, k1 + u);
#pragma unroll
        for (int i = 0; i < 8; i++) fb[u][i] = al_ld(k1 + u, i);
      }
      tbl8(k1, ft);
    };
    fetch(M, nx, nb, nt);
    for (int g = 0; g < (K - M) / P; g++) {
      const int k0 = M + g * P;
      StepIn cs[P];
      s2 cb[P][8];
      int ct[P];
#pragma unroll
      for (int u = 0; u < P; u++) {
        cs[u] = nx[u];
        ct[u] = nt[u];
#pragma unroll
        for (int i = 0; i < 8; i++) cb[u][i] = nb[u][i];
      }
      fetch(min(k0 + P, K - P), nx, nb, nt);
#pragma unroll
      for (int u = 0; u < P; u++) {
        const int k = k0 + u;
        const StepIn &st = cs[u];
        const s2 g1 = wadd(st.x, st.y) >> 1, g0 = wsub(st.x, st.y) >> 1;
        s2 bp[8], bn[8];
        bpn(cb[u], g0, g1, bp, bn);
        const s2 llr = llr_of(bp, bn, apre);
        out_st(ct[u], llr, st.e);
        if (dout) { // k ascends: flush each 16-step group at its last step (M and K multiples of 8)
          dacc |= dec_bits(llr) << (k & 15);
          if (u == P - 1 && ((k & 15) == 15 || k == K - 1)) {
            bst32s(dacc, R.d, R.vd, (uint32_t)(k >> 4) * 4);
            dacc = 0;
          }
        }
        s2 n[8];
        astep(a, g0, g1, n);
#pragma unroll
        for (int i = 0; i < 8; i++) {
          a[i] = n[i];
          apre[i] = n[i];
        }
        if ((u & 3) == 3) norm(a);
      }
    }
    return;
  }
  s2 b[8];
  b[0] = splat(0);
#pragma unroll
  for (int i = 1; i < 8; i++) b[i] = splat(-TD_INF);
  if (!done) { // phase 1: tail steps K+2..K (C-division gammas, :349-352), then betas K-1..M
    const int tail_xoff = MODE == 1 ? 6 : 0;
    for (int k = K + 2; k >= K; k--) {
      const s2 x = tl[tail_xoff + 2 * (k - K)], y = tl[tail_xoff + 2 * (k - K) + 1];
      const s2 g0 = s2{(short)(((int)x.x - y.x) / 2), (short)(((int)x.y - y.y) / 2)};
      const s2 g1 = s2{(short)(((int)x.x + y.x) / 2), (short)(((int)x.y + y.y) / 2)};
      s2 bp[8], bn[8];
      bpn(b, g0, g1, bp, bn);
#pragma unroll
      for (int i = 0; i < 8; i++) b[i] = smax(bp[i], bn[i]);
    }
    StepIn nx[P];
#pragma unroll
    for (int u = 0; u < P; u++) nx[u] = sse_ld<MODE>(R, K - 1 - u);
    for (int g = 0; g < (K - M) / P; g++) {
      const int k1 = K - 1 - g * P; // k1 - u = 8 j + 7 - u: (k & 3) == 0 at u = 3, 7
      StepIn cu[P];
#pragma unroll
      for (int u = 0; u < P; u++) cu[u] = nx[u];
#pragma unroll
      for (int u = 0; u < P; u++) nx[u] = sse_ld<MODE>(R, k1 - P - u); // >= M - 8 >= 8
#pragma unroll
      for (int u = 0; u < P; u++) {
        const int k = k1 - u;
#pragma unroll
        for (int i = 0; i < 8; i++) al_st(k, i, b[i]); // B(k)
        const s2 g1 = wadd(cu[u].x, cu[u].y) >> 1, g0 = wsub(cu[u].x, cu[u].y) >> 1;
        s2 bp[8], bn[8];
        bpn(b, g0, g1, bp, bn);
#pragma unroll
        for (int i = 0; i < 8; i++) b[i] = smax(bp[i], bn[i]);
        if ((u & 3) == 3) norm(b);
      }
    }
  }
  __syncthreads();
  if (done) return;
  // phase 2: betas and LLRs of steps M-1..0 from the stored alphas
  StepIn ns[P];
  s2 na[P][8];
  int nt[P];
  auto fetchb = [&](int k1, StepIn *fs, s2 (*fa)[8], int *ft) {
#pragma unroll
    for (int u = 0; u < P; u++) {
      fs[u] = sse_ld<MODE>(R, k1 - u);
#pragma unroll
      for (int i = 0; i < 8; i++) fa[u][i] = al_ld(k1 - u, i);
    }
    int t8[8];
    tbl8(k1 - (P - 1), t8);
#pragma unroll
    for (int u = 0; u < P; u++) ft[u] = t8[P - 1 - u];
  };
  fetchb(M - 1, ns, na, nt);
  for (int g = 0; g < M / P; g++) {
    const int k1 = M - 1 - g * P;
    StepIn cs[P];
    s2 ca[P][8];
    int ct[P];
#pragma unroll
    for (int u = 0; u < P; u++) {
      cs[u] = ns[u];
      ct[u] = nt[u];
#pragma unroll
      for (int i = 0; i < 8; i++) ca[u][i] = na[u][i];
    }
    fetchb(max(k1 - P, P - 1), ns, na, nt);
#pragma unroll
    for (int u = 0; u < P; u++) {
      const int k = k1 - u;
      const StepIn &st = cs[u];
      const s2 g1 = wadd(st.x, st.y) >> 1, g0 = wsub(st.x, st.y) >> 1;
      s2 bp[8], bn[8];
      bpn(b, g0, g1, bp, bn);
#pragma unroll
      for (int i = 0; i < 8; i++) b[i] = smax(bp[i], bn[i]);
      const s2 llr = llr_of(bp, bn, ca[u]);
      out_st(ct[u], llr, st.e);
      if (dout) { // k descends: flush each 16-step group at its first step
        dacc |= dec_bits(llr) << (k & 15);
        if (u == P - 1 && (k & 15) == 0) {
          bst32s(dacc, R.d, R.vd, (uint32_t)(k >> 4) * 4);
          dacc = 0;
        }
      }
      if ((u & 3) == 3) norm(b);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(128) void k_sse_bidir(const TdGroup *__restrict__ groups, int ngroups,
                                                   const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                   s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                   const s2 *__restrict__ T, size_t plane,
                                                   s2 *__restrict__ scratch_base,
                                                   const uint8_t *__restrict__ pair_done) {
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int p = (blockIdx.x - G.blk_half) * 64 + (threadIdx.x & 63);
  const bool done = p >= G.npairs || (pair_done && pair_done[G.pair0 + p]);
  sse_bidir_body<MODE>(G, p, done, SP0, XP1, Aarr, Darr, T, plane, scratch_base);
}

// The early stop of the SSE decoder after half-iteration n, as es_check does it for the window
// kernels (CRC as the XOR of the weights TdGroup::wc over the set decision bits, crc.c:144-155;
// the done / ok / noi update of sch.c:361-391; the decision words of the blocks ending now kept
// for k_es_bytes), one pair per lane: each wave folds the decision words it wrote (wave 1 those
// below M / 16, wave 0 the rest), wave 0 combines, decides and keeps the words.
// fin[2 lane + h]: bit 0 = done, bit 1 = ended at this check. Returns (uniformly) whether every
// pair of the workgroup is done.
template <int V = 0> // a template so that only the part that launches k_sse_es instantiates it
__device__ __noinline__ bool sse_es_check(const TdGroup &G, int p, int n, const uint32_t *__restrict__ Darr,
                                          const TdEs &es, uint32_t *red, int *fin) {
  const int K = G.K, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nw = dec_words(K, 1), mw = (16 * (K / 32)) / 16;
  const bool dec2 = n & 1;
  const bool live = !((fin[2 * lane] & 1) && (fin[2 * lane + 1] & 1));
  const int pair = p < G.npairs ? p : G.npairs - 1;
  const gptr_t<uint32_t> dw = gptr(Darr + G.dw0 + (size_t)pair * nw);
  uint32_t c0 = 0, c1 = 0;
  if (live) {
    const gptr_t<uint32_t> wc = gptr(G.wc[dec2 ? 1 : 0]);
    const int q0 = wv ? 0 : mw, q1 = wv ? mw : nw;
    for (int q = q0; q < q1; q++) {
      const uint32_t w = dw[q];
      if (w == 0u) continue;
      const gptr_t<u4> wq = (gptr_t<u4>)(wc + (size_t)q * 16);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const u4 v = wq[i];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int b = 4 * i + j;
          c0 ^= ((w >> b) & 1u) ? v[j] : 0u;
          c1 ^= ((w >> (16 + b)) & 1u) ? v[j] : 0u;
        }
      }
    }
  }
  if (wv) {
    red[2 * lane] = c0;
    red[2 * lane + 1] = c1;
  }
  __syncthreads();
  if (!wv) {
    const uint32_t crc[2] = {c0 ^ red[2 * lane], c1 ^ red[2 * lane + 1]};
#pragma unroll
    for (int h = 0; h < 2; h++) {
      int f = fin[2 * lane + h] & 1;
      if (!f) {
        const int cb = G.cb0 + 2 * p + h;
        es.noi[cb] = (uint32_t)(n + 1);
        if (crc[h] == 0u) {
          es.cb_ok[cb] = 1;
          es.cb_done[cb] = 1;
          f = 3;
        } else if (n + 1 >= es.max_halfits) {
          es.cb_done[cb] = 1;
          f = 3;
        }
      }
      fin[2 * lane + h] = f & 1 ? f : 0;
    }
  }
  if (!wv) { // blocks that ended now: their decision words into Dfz, parity into cb_end (es_check)
    const int f0 = fin[2 * lane], f1 = fin[2 * lane + 1];
    const uint32_t mask = ((f0 & 2) ? 0xffffu : 0u) | ((f1 & 2) ? 0xffff0000u : 0u);
    if (mask) {
      const gmut_t<uint32_t> fz = gmut<uint32_t>(es.dfz + G.dw0 + (size_t)pair * nw);
      for (int q = 0; q < nw; q++) fz[q] = (fz[q] & ~mask) | (dw[q] & mask);
      if (f0 & 2) es.cb_end[G.cb0 + 2 * p] = (uint8_t)(1 + (n & 1));
      if (f1 & 2) es.cb_end[G.cb0 + 2 * p + 1] = (uint8_t)(1 + (n & 1));
    }
  }
  __syncthreads();
  return __syncthreads_and((fin[2 * lane] & 1) && (fin[2 * lane + 1] & 1));
}

// The early-stop form of the SSE decoder (the DL-SCH path for K <= 400 under AUTO): up to
// max_halfits half-iterations of k_sse_bidir in ONE launch, each followed by sse_es_check; the
// workgroup leaves once all of its pairs are done, a finished pair's lanes idle through the rest.
// Blocks done at entry (HARQ retransmissions whose CRC passed before) are seeded from cb_done.
template <int V = 0>
__global__ __launch_bounds__(128) void k_sse_es(const TdGroup *__restrict__ groups, int ngroups,
                                                const s4 *__restrict__ SP0, s2 *__restrict__ XP1,
                                                s2 *__restrict__ Aarr, uint32_t *__restrict__ Darr,
                                                const s2 *__restrict__ T, size_t plane,
                                                s2 *__restrict__ scratch_base, TdEs es) {
  __shared__ uint32_t red[128];
  __shared__ int fin[128];
  wave_prio(es.prio);
  const TdGroup &G = groups[grp_find<GF_HALF>(groups, ngroups, blockIdx.x)];
  const int p = (blockIdx.x - G.blk_half) * 64 + (threadIdx.x & 63);
  if (threadIdx.x < 64) {
#pragma unroll
    for (int h = 0; h < 2; h++)
      fin[2 * threadIdx.x + h] =
          (p >= G.npairs || 2 * p + h >= G.ncb || es.cb_done[G.cb0 + 2 * p + h]) ? 1 : 0;
  }
  __syncthreads();
  if (__syncthreads_and((fin[2 * (threadIdx.x & 63)] & 1) && (fin[2 * (threadIdx.x & 63) + 1] & 1)))
    return;
  for (int n = es.n0; n < es.n1; n++) {
    const int l = threadIdx.x & 63;
    const bool done = (fin[2 * l] & 1) && (fin[2 * l + 1] & 1);
    if (n & 1)
      sse_bidir_body<1>(G, p, done, SP0, XP1, Aarr, Darr, T, plane, scratch_base);
    else if (n == 0)
      sse_bidir_body<2>(G, p, done, SP0, XP1, Aarr, Darr, T, plane, scratch_base);
    else
      sse_bidir_body<0>(G, p, done, SP0, XP1, Aarr, Darr, T, plane, scratch_base);
    __syncthreads(); // both waves' decision words and outputs of the half-iteration are written
    if (sse_es_check<V>(G, p, n, Darr, es, red, fin)) break;
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
  const size_t base = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, 1);
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
#if TD_PART == 0 // loaders, decide: part 0 only
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
  // the tile's steps k0 .. k0+kn-1 of all NB chains are one contiguous T4 run from k0 * NB
  // (k0 is a multiple of 4), written in order: e -> step (e / 4 / NB) * 4 + e % 4, chain e / 4 % NB
  const size_t base = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, NB) + (size_t)k0 * NB;
  const int ne = ((kn + 3) >> 2) * NB * 4;
  for (int e = threadIdx.x; e < ne; e += 256) {
    const int gq = e >> 2, kk = (gq / NB) * 4 + (e & 3), dd = gq - (gq / NB) * NB;
    if (kk >= kn) continue;
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
  const int nb = G.nb;
  const size_t o0 = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, nb);
#pragma unroll
  for (int u = 0; u < 2; u++) { // SB index i + u = step k, chain d -> T4 position
    const int k = (i + u) / nb, dd = (i + u) - k * nb;
    const size_t o = o0 + t4_pos(k, dd, nb);
    SP0[o] = s4{a[i + u], b[i + u], a[K + 32 + i + u], b[K + 32 + i + u]};
    P1[o] = s2{a[2 * (K + 32) + i + u], b[2 * (K + 32) + i + u]};
  }
  if (i < 12) {
    const int tb = 3 * (K + 32);
    const size_t t = (size_t)(G.pair0 + pair) * 12 + i;
    T[t] = s2{a[tb + i], b[tb + i]};
    T[t + 1] = s2{a[tb + i + 1], b[tb + i + 1]};
  }
}

// The same copy for 16-byte aligned rows (the DL-SCH softbuffer rows; K a multiple of 8, so
// chains pair up), one T4 group (4 steps) of two adjacent chains d, d+1 of a pair per thread:
// 4-byte loads of the two chains' values per step and stream (consecutive threads read
// consecutive chain pairs), then the two chains' 32-byte SP0 groups and 16-byte P1 groups, which
// are adjacent in T4, as 16-byte stores.
__global__ __launch_bounds__(256) void k_load_sb8(const TdGroup *__restrict__ groups, int ngroups,
                                                  const int16_t *__restrict__ in, size_t in_stride,
                                                  const int16_t *const *__restrict__ rows,
                                                  TdArrays arr) {
  const TdGroup &G = groups[grp_find<GF_LOAD>(groups, ngroups, blockIdx.x)];
  const int K = G.K, ncb = G.ncb, npairs = G.npairs, nb = G.nb;
  const int L = K / nb, G4 = (L + 3) >> 2, hp = nb >> 1;
  const int per = G4 * hp;
  const size_t gid = (size_t)(blockIdx.x - G.blk_load) * 256 + threadIdx.x;
  const int pair = (int)(gid / per);
  if (pair >= npairs) return;
  const int r = (int)(gid - (size_t)pair * per);
  const int g4 = r / hp, d = 2 * (r - g4 * hp);
  const int c0 = G.cb0 + 2 * pair, c1 = 2 * pair + 1 < ncb ? c0 + 1 : c0;
  const gptr_t<int16_t> a = cb_row(in, in_stride, rows, c0), b = cb_row(in, in_stride, rows, c1);
  auto ld2 = [](gptr_t<int16_t> p) { return *(const __attribute__((address_space(1))) uint32_t *)p; };
  uint32_t sa[4], sb[4], pa[4], pb[4], qa[4], qb[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {
    const int k = min(4 * g4 + u, L - 1); // the last group may run past L: values unused
    const int i = k * nb + d;             // even: 4-byte aligned
    sa[u] = ld2(a + i);
    sb[u] = ld2(b + i);
    pa[u] = ld2(a + K + 32 + i);
    pb[u] = ld2(b + K + 32 + i);
    qa[u] = ld2(a + 2 * (K + 32) + i);
    qb[u] = ld2(b + 2 * (K + 32) + i);
  }
  // chain h (0: d, 1: d + 1) of CB x / y: low / high half of the loaded words
  auto lo = [](uint32_t x, uint32_t y) { return (x & 0xffffu) | (y << 16); };
  auto hi = [](uint32_t x, uint32_t y) { return (x >> 16) | (y & 0xffff0000u); };
  const size_t o = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, nb) + (size_t)(g4 * nb + d) * 4;
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  const gmut_t<u4v> SP0 = gmut<u4v>((s4 *)arr.SP0 + o); // 2 chains x 4 steps x 8 B: four u4v
  const gmut_t<u4v> P1 = gmut<u4v>((s2 *)arr.XP1 + arr.plane + o); // 2 x 4 x 4 B: two u4v
#pragma unroll
  for (int h = 0; h < 2; h++) {
    auto f = [&](uint32_t x, uint32_t y) { return h ? hi(x, y) : lo(x, y); };
    SP0[2 * h] = u4v{f(sa[0], sb[0]), f(pa[0], pb[0]), f(sa[1], sb[1]), f(pa[1], pb[1])};
    SP0[2 * h + 1] = u4v{f(sa[2], sb[2]), f(pa[2], pb[2]), f(sa[3], sb[3]), f(pa[3], pb[3])};
    P1[h] = u4v{f(qa[0], qb[0]), f(qa[1], qb[1]), f(qa[2], qb[2]), f(qa[3], qb[3])};
  }
  if (r == 0) { // one thread per pair: the tails
    const int tb = 3 * (K + 32);
    const gmut_t<s2> T = gmut<s2>(arr.T);
#pragma unroll
    for (int t = 0; t < 12; t++) T[(size_t)(G.pair0 + pair) * 12 + t] = s2{a[tb + t], b[tb + t]};
  }
}

// The same copy through LDS for nb a multiple of 8 (the window decoders' rows): a workgroup takes
// 1024 / nb steps of one pair (2 KB per CB and stream), loads its 6 chunks with coalesced 16-byte
// loads (3 per thread), and writes the steps' SP0 (8 KB) and P1 (4 KB) T4 tiles, which are
// contiguous, with coalesced 16-byte stores (3 per thread). The per-thread forms read and write
// 16-byte pieces whose neighbours belong to other instructions.
#define LSBT_STEPS(nb) (1024 / (nb))
__global__ __launch_bounds__(256) void k_load_sbt(const TdGroup *__restrict__ groups, int ngroups,
                                                  const int16_t *__restrict__ in, size_t in_stride,
                                                  const int16_t *const *__restrict__ rows,
                                                  TdArrays arr) {
  __shared__ uint16_t lds[6][1024];
  const TdGroup &G = groups[grp_find<GF_LOAD>(groups, ngroups, blockIdx.x)];
  const int K = G.K, ncb = G.ncb, npairs = G.npairs, nb = G.nb;
  const int L = K / nb, G4 = (L + 3) >> 2, S = LSBT_STEPS(nb);
  const int per = (4 * G4 + S - 1) / S; // workgroups per pair
  const int w = blockIdx.x - G.blk_load;
  const int pair = w / per, ch = w - pair * per;
  if (pair >= npairs) return;
  const int k0 = ch * S;
  const int c0 = G.cb0 + 2 * pair, c1 = 2 * pair + 1 < ncb ? c0 + 1 : c0;
  const gptr_t<int16_t> rw[2] = {cb_row(in, in_stride, rows, c0), cb_row(in, in_stride, rows, c1)};
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int q = 0; q < 3; q++) {
    const int idx = threadIdx.x + 256 * q; // 6 chunks x 128 pieces of 8 elements
    const int c = idx >> 7, piece = idx & 127;
    const int st = c >> 1, h = c & 1; // stream (sys, p0, p1), CB
    int e = k0 * nb + piece * 8;      // element in the stream; past the last step: its copy
    if (e >= L * nb) e = (L - 1) * nb + (e & (nb - 1));
    const u4v v = *(const __attribute__((address_space(1))) u4v *)(rw[h] + st * (K + 32) + e);
    *(u4v *)&lds[c][piece * 8] = v;
  }
  __syncthreads();
  const size_t e0 = (size_t)G.elem0 + (size_t)pair * t4_pair_elems(K, nb) + (size_t)k0 * nb;
  const int nel = min(S, 4 * G4 - k0) * nb; // T4 elements of this tile (the pair's padded steps)
  auto at = [&](int c, int el) -> uint32_t { // T4 element el of the tile -> stream value
    const int g4l = el / (4 * nb), d = (el >> 2) % nb, u = el & 3;
    return lds[c][(4 * g4l + u) * nb + d];
  };
  const gmut_t<u4v> SP0 = gmut<u4v>((s4 *)arr.SP0 + e0);
  const gmut_t<u4v> P1 = gmut<u4v>((s2 *)arr.XP1 + arr.plane + e0);
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const int v = threadIdx.x + 256 * q; // SP0 elements 2v, 2v + 1
    if (2 * v >= nel) break;
    const int ea = 2 * v, eb = 2 * v + 1;
    SP0[v] = u4v{at(0, ea) | (at(1, ea) << 16), at(2, ea) | (at(3, ea) << 16),
                 at(0, eb) | (at(1, eb) << 16), at(2, eb) | (at(3, eb) << 16)};
  }
  if (4 * (int)threadIdx.x < nel) {
    const int e = 4 * threadIdx.x;
    P1[threadIdx.x] = u4v{at(4, e) | (at(5, e) << 16), at(4, e + 1) | (at(5, e + 1) << 16),
                          at(4, e + 2) | (at(5, e + 2) << 16), at(4, e + 3) | (at(5, e + 3) << 16)};
  }
  if (ch == 0 && threadIdx.x < 12) { // the tails
    const int tb = 3 * (K + 32), t = threadIdx.x;
    gmut<s2>(arr.T)[(size_t)(G.pair0 + pair) * 12 + t] = s2{rw[0][tb + t], rw[1][tb + t]};
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
                                                int max_halfits, uint8_t *__restrict__ pair_done, int prio,
                                                uint32_t *__restrict__ run_list, uint32_t *__restrict__ run_cnt,
                                                int knobs_dev_word_bytes) {
  __shared__ uint32_t dw[6144 / 16 + 16];
  __shared__ uint32_t red[2][4];
  __shared__ int fin[4]; // [0..1] CB done, [2..3] CB finished at this half-iteration
  wave_prio(prio);
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
    if (threadIdx.x == 0 && run_list && !(fin[0] && fin[1])) // still running: into the group's list
      run_list[G.pair0 + atomicAdd(&run_cnt[G.pair0], 1u)] = (uint32_t)pair;
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
  if (!dec2 && knobs_dev_word_bytes) {
    // after DEC1 a byte inside one chain is 8 consecutive bits of its chain: each thread forms whole
    // 32-bit output words from the staged words (h0_byte), one store per word
    const int nbytes = K / 8, nwd = nbytes / 4;
    const bool w32 = ((uintptr_t)outb & 3u) == 0 && (out_stride & 3u) == 0;
    for (int h = 0; h < 2; h++) {
      if (!out[h]) continue;
      uint8_t *row = outb + (size_t)cbs[h] * out_stride;
      if (w32) {
        for (int w = threadIdx.x; w < nwd; w += blockDim.x) {
          const int p = 32 * w;
          reinterpret_cast<uint32_t *>(row)[w] =
              h0_byte(dw, nw, L, gap, invL, h, p) | (h0_byte(dw, nw, L, gap, invL, h, p + 8) << 8) |
              (h0_byte(dw, nw, L, gap, invL, h, p + 16) << 16) | (h0_byte(dw, nw, L, gap, invL, h, p + 24) << 24);
        }
        for (int b = 4 * nwd + (int)threadIdx.x; b < nbytes; b += blockDim.x)
          row[b] = (uint8_t)h0_byte(dw, nw, L, gap, invL, h, 8 * b);
      } else {
        for (int b = threadIdx.x; b < nbytes; b += blockDim.x) row[b] = (uint8_t)h0_byte(dw, nw, L, gap, invL, h, 8 * b);
      }
    }
    return;
  }
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

// Natural-order bytes of the blocks a fused early-stop decode ended (es_check / sse_es_check kept
// their decision words in Dfz and 1 + the parity of the ending half-iteration in cb_end), as
// k_decide writes them (turbodecoder.c:353-360 + decision_byte, MSB first); one workgroup per CB
// pair, many pairs in flight. Clears cb_end behind it.
#define ESB_PAIRS 8 // pairs per workgroup: most pairs of a batch ended before the fused launch
__global__ __launch_bounds__(256) void k_es_bytes(const TdGroup *__restrict__ groups, int ngroups, int npairs_total,
                                                  const uint32_t *__restrict__ Dfz,
                                                  uint8_t *__restrict__ outb, size_t out_stride,
                                                  uint8_t *__restrict__ cb_end, int prio) {
  __shared__ uint32_t dw[6144 / 16 + 16];
  __shared__ int todo[ESB_PAIRS], ntodo;
  wave_prio(prio);
  // the workgroup's pairs' flags all at once (one thread per pair), then only the pairs that ended
  // (a pair-by-pair scan waited on two dependent loads per pair, ~45 us per launch)
  if (threadIdx.x == 0) ntodo = 0;
  __syncthreads();
  if (threadIdx.x < ESB_PAIRS) {
    const int gp = blockIdx.x * ESB_PAIRS + threadIdx.x;
    if (gp < npairs_total) {
      const TdGroup &G = groups[grp_find<GF_PAIR>(groups, ngroups, gp)];
      const int pair = gp - G.pair0;
      if (pair < G.npairs) {
        const int c0 = G.cb0 + 2 * pair;
        if (cb_end[c0] || (2 * pair + 1 < G.ncb && cb_end[c0 + 1])) todo[atomicAdd(&ntodo, 1)] = gp;
      }
    }
  }
  __syncthreads();
  const int nt = ntodo;
  for (int ti = 0; ti < nt; ti++) {
  const int gp = todo[ti];
  const TdGroup &G = groups[grp_find<GF_PAIR>(groups, ngroups, gp)];
  const int K = G.K, NB = G.nb, ncb = G.ncb;
  const int pair = gp - G.pair0;
  const int cbs[2] = {G.cb0 + 2 * pair, 2 * pair + 1 < ncb ? G.cb0 + 2 * pair + 1 : -1};
  const int ends[2] = {cb_end[cbs[0]], cbs[1] >= 0 ? cb_end[cbs[1]] : 0};
  const int L = K / NB, G16 = (L + 15) / 16, nw = NB * G16;
  const uint32_t *src = Dfz + G.dw0 + (size_t)pair * nw;
  for (int q = threadIdx.x; q < nw; q += blockDim.x) dw[q] = src[q];
  __syncthreads();
  const gptr_t<uint16_t> dmap = gptr(G.dmap);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float invL = 1.0f / (float)L;
  const int gap = 16 * G16 - L;
  constexpr int PMAX = 6144 / 256;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (!ends[h]) continue;
    const bool dec2 = ends[h] == 2;
    int ci[PMAX];
#pragma unroll
    for (int u = 0; u < PMAX; u++) { // every map load issued before the first use
      const int p = wv * 64 + u * 256 + lane;
      int c = 0;
      if (p < K) {
        if (dec2) {
          c = (int)dmap[p];
        } else {
          const int d = (int)(((float)p + 0.5f) * invL);
          c = p + d * gap;
        }
      }
      ci[u] = c;
    }
    uint8_t *ob = outb + (size_t)cbs[h] * out_stride;
#pragma unroll
    for (int u = 0; u < PMAX; u++) {
      const int p0 = wv * 64 + u * 256;
      if (p0 >= K) break;
      const int p = p0 + lane;
      const uint32_t bit = p < K ? (dw[ci[u] >> 4] >> ((ci[u] & 15) + 16 * h)) & 1u : 0u;
      const uint64_t m = __ballot(bit);
      if (lane < 8 && p0 + 8 * lane < K) {
        const uint32_t v = (uint32_t)((m >> (8 * lane)) & 0xffu);
        ob[(p0 >> 3) + lane] = (uint8_t)(__builtin_bitreverse32(v) >> 24);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 && cbs[threadIdx.x] >= 0) cb_end[cbs[threadIdx.x]] = 0;
  }
}

// The early-stop flags of the job's code blocks, one thread per pair: done = init_done (blocks
// decoded in an earlier transmission; none without init_done), ok = 0, noi = 0, and pair_done =
// both blocks done. One launch instead of two fills, a copy and the pair pass.
__global__ void k_pair_done(const TdGroup *__restrict__ groups, int ngroups, int npairs_total,
                            const uint8_t *__restrict__ init_done, uint8_t *__restrict__ cb_done,
                            uint8_t *__restrict__ cb_ok, uint32_t *__restrict__ noi,
                            uint8_t *__restrict__ pair_done, uint32_t *__restrict__ run_cnt) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs_total) return;
  if (run_cnt) run_cnt[p] = 0; // the groups' running-pair counts (at their pair0)
  const TdGroup &G = groups[grp_find<GF_PAIR>(groups, ngroups, p)];
  const int lp = p - G.pair0;
  const int c0 = G.cb0 + 2 * lp, c1 = 2 * lp + 1 < G.ncb ? c0 + 1 : c0;
  const uint8_t d0 = init_done ? init_done[c0] : 0, d1 = init_done ? init_done[c1] : 0;
  cb_done[c0] = d0;
  cb_ok[c0] = 0;
  noi[c0] = 0;
  cb_done[c1] = d1;
  cb_ok[c1] = 0;
  noi[c1] = 0;
  pair_done[p] = d0 && d1;
}

#endif // TD_PART == 0

// ------------------------------------------------------------------ launchers ----

static inline unsigned nblk(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// dynamic LDS above 64 KiB (the 8-sub-block decoder at large K) needs the per-kernel opt-in
[[maybe_unused]] static void allow_big_lds(const void *f, int static_bytes = 0) {
  const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - static_bytes);
  if (e != hipSuccess) fprintf(stderr, "srsgpu: dynamic LDS opt-in failed: %s\n", hipGetErrorString(e));
}

#if TD_PART == 0
int load_blocks(int K, int nb, int npairs, int sb_input, bool vec16) {
  if (sb_input && vec16)
    return nb % 8 == 0 ? npairs * ((4 * ((K / nb + 3) / 4) + 1024 / nb - 1) / (1024 / nb))
                       : (int)nblk((size_t)npairs * ((K / nb + 3) / 4) * (nb / 2), 256);
  if (sb_input) return (int)nblk((size_t)npairs * (K / 2), 256);
  return npairs * ((K / nb + LOAD_KT - 1) / LOAD_KT);
}

int halfit_blocks(int nb, int npairs) { return nb > 1 ? (int)nblk((size_t)npairs * nb, 64) : (int)nblk(npairs, 64); }

size_t seq_scratch_elems(int K, int npairs) { return (size_t)(K + 4) * 8 * npairs; }


size_t bidir_lds_bytes(int K, int nb) {
#ifdef TD_EXP_HALFLDS
  return (size_t)(((K / nb + TD_BIDIR_CW - 1) / TD_BIDIR_CW + 1) / 2 + 1) * 2 * 64 * 16;
#endif
  return (size_t)((K / nb + TD_BIDIR_CW - 1) / TD_BIDIR_CW + 1) * 2 * 64 * 16;
}

int dec_words_host(int K, int nb) { return nb * ((K / nb + 15) / 16); }

hipError_t launch_load(const TdGroup *dg, int ng, int nblocks, int nb, int sb_input, bool vec,
                       const int16_t *in, size_t in_stride, const int16_t *const *rows,
                       const TdArrays &a, hipStream_t st) {
  if (ng <= 0 || nblocks <= 0) return hipSuccess;
  if (sb_input) {
    if (vec && nb % 8 == 0) // 16-byte aligned rows, LDS-transposed tiles (load_blocks counted tiles)
      hipLaunchKernelGGL(k_load_sbt, dim3(nblocks), dim3(256), 0, st, dg, ng, in, in_stride, rows, a);
    else if (vec) // 16-byte aligned rows (load_blocks counted 8 elements per thread)
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

#endif // TD_PART == 0

// Kernel instances by part, so the library builds in parallel translation units (each part
// file defines TD_PART and includes this file): part 0 = loaders, decide and the dispatchers
// below; parts 1-4 = the window decoders of one kind each (per-half-iteration and fused), part 2
// also the sequential decoders.
// one decoder kind's per-half-iteration (halfit_part) and fused (halfits_part) launchers,
// specialised in the part that instantiates the kind
template <int KIND>
hipError_t halfit_part(int mode, const TdGroup *dg, int ng, int nblocks, size_t lds, bool dec,
                       const TdArrays &a, const uint8_t *pair_done, hipStream_t st);
template <int KIND>
hipError_t halfits_part(int n0, int nh, const TdGroup *dg, int ng, int nblocks, size_t lds, bool dec,
                        const TdArrays &a, hipStream_t st);
template <int KIND>
hipError_t halfits_es_part(const TdGroup *dg, int ng, int nblocks, size_t lds, const TdArrays &a,
                           const TdEs &es, hipStream_t st);

#define BIDIR1(nb, div, m, dout, b8)                                                               \
  do {                                                                                             \
    allow_big_lds((const void *)(k_win_bidir<nb, div, m, TD_BIDIR_CW, dout, b8>));                 \
    hipLaunchKernelGGL((k_win_bidir<nb, div, m, TD_BIDIR_CW, dout, b8>), dim3(nblocks), dim3(128), \
                       lds, st, dg, ng, (const s4 *)a.SP0, (s2 *)a.XP1, (s2 *)a.A,               \
                       (uint32_t *)a.D, (const s2 *)a.T, a.plane, pair_done,                      \
                       knobs().h0_prio);                                              \
  } while (0)
#define BIDIR(nb, div, b8)                                                                         \
  do {                                                                                             \
    if (mode == 1) {                                                                               \
      if (dec) BIDIR1(nb, div, 1, true, b8); else BIDIR1(nb, div, 1, false, b8);                   \
    } else if (mode == 2) {                                                                        \
      if (dec) BIDIR1(nb, div, 2, true, b8); else BIDIR1(nb, div, 2, false, b8);                   \
    } else {                                                                                       \
      if (dec) BIDIR1(nb, div, 0, true, b8); else BIDIR1(nb, div, 0, false, b8);                   \
    }                                                                                              \
  } while (0)
#define SEQT(kern, nt)                                                                             \
  do {                                                                                             \
    if (mode == 1) SEQ1(kern, 1, nt); else if (mode == 2) SEQ1(kern, 2, nt); else SEQ1(kern, 0, nt); \
  } while (0)
#define SEQ(kern) SEQT(kern, 64)
#define SEQ1(kern, m, nt)                                                                          \
  hipLaunchKernelGGL(kern<m>, dim3(nblocks), dim3(nt), 0, st, dg, ng, (const s4 *)a.SP0,            \
                     (s2 *)a.XP1, (s2 *)a.A, (uint32_t *)a.D, (const s2 *)a.T, a.plane,             \
                     (s2 *)a.scratch, pair_done)
#define RUN1(nb, div, b8)                                                                          \
  do {                                                                                             \
    allow_big_lds((const void *)(k_win_bidir_run<nb, div, b8>));                                   \
    hipLaunchKernelGGL((k_win_bidir_run<nb, div, b8>), dim3(nblocks), dim3(128), lds, st, dg, ng,  \
                       (const s4 *)a.SP0, (s2 *)a.XP1, (s2 *)a.A, (uint32_t *)a.D,                 \
                       (const s2 *)a.T, a.plane, n0, nh, dec ? 1 : 0);                             \
  } while (0)
#define RUNES(nb, div, b8)                                                                         \
  do {                                                                                             \
    if (es.bytes_direct && es.n0 == 0 && es.n1 == 1) { /* first half-iteration + its check */      \
      allow_big_lds((const void *)(k_win_bidir_h0c<nb, div, b8>), 1024);                           \
      hipLaunchKernelGGL((k_win_bidir_h0c<nb, div, b8>), dim3(nblocks), dim3(128), lds, st, dg, ng, \
                         (const s4 *)a.SP0, (s2 *)a.XP1, (s2 *)a.A, (uint32_t *)a.D,               \
                         (const s2 *)a.T, a.plane, es);                                            \
      break;                                                                                       \
    }                                                                                              \
    allow_big_lds((const void *)(k_win_bidir_es<nb, div, b8>), 1024); /* + its static LDS */       \
    hipLaunchKernelGGL((k_win_bidir_es<nb, div, b8>), dim3(nblocks), dim3(128), lds, st, dg, ng,   \
                       (const s4 *)a.SP0, (s2 *)a.XP1, (s2 *)a.A, (uint32_t *)a.D,                 \
                       (const s2 *)a.T, a.plane, es);                                              \
  } while (0)
#define PART_FUNCS(KIND, HALFIT_BODY, RUN_BODY, ES_BODY)                                           \
  template <>                                                                                      \
  hipError_t halfit_part<KIND>(int mode, const TdGroup *dg, int ng, int nblocks, size_t lds,       \
                               bool dec, const TdArrays &a, const uint8_t *pair_done,              \
                               hipStream_t st) {                                                   \
    HALFIT_BODY;                                                                                   \
    return hipGetLastError();                                                                      \
  }                                                                                                \
  template <>                                                                                      \
  hipError_t halfits_part<KIND>(int n0, int nh, const TdGroup *dg, int ng, int nblocks, size_t lds, \
                                bool dec, const TdArrays &a, hipStream_t st) {                     \
    RUN_BODY;                                                                                      \
    return hipGetLastError();                                                                      \
  }                                                                                                \
  template <>                                                                                      \
  hipError_t halfits_es_part<KIND>(const TdGroup *dg, int ng, int nblocks, size_t lds,             \
                                   const TdArrays &a, const TdEs &es, hipStream_t st) {            \
    ES_BODY;                                                                                       \
    return hipGetLastError();                                                                      \
  }

// k_win_spread launchers, one per windowed kind (in the part that holds the kind)
template <int KIND>
hipError_t spread_part(int mode, const TdGroup *dg, int npairs, size_t lds, bool dec, const TdArrays &a,
                       const uint8_t *pair_done, uint8_t *outb, size_t out_stride, const SpreadOut &so,
                       hipStream_t st);
#define SPREAD1(nb, div, m, dout, b8)                                                              \
  hipLaunchKernelGGL((k_win_spread<nb, div, m, dout, b8>), dim3(npairs * TD_SPREAD_SPLIT),           \
                     dim3(TD_SPREAD_THREADS), lds, st, dg, (const s4 *)a.SP0, (s2 *)a.XP1, (s2 *)a.A, \
                     (uint32_t *)a.D, (const s2 *)a.T, a.plane, pair_done, outb, out_stride, so.cnt, \
                     so.flag, so.seq)
#define SPREAD(KIND, nb, div, b8)                                                                  \
  template <>                                                                                      \
  hipError_t spread_part<KIND>(int mode, const TdGroup *dg, int npairs, size_t lds, bool dec,      \
                               const TdArrays &a, const uint8_t *pair_done, uint8_t *outb,         \
                               size_t out_stride, const SpreadOut &so, hipStream_t st) {          \
    if (mode == 1) {                                                                               \
      if (dec) SPREAD1(nb, div, 1, true, b8); else SPREAD1(nb, div, 1, false, b8);                 \
    } else if (mode == 2) {                                                                        \
      if (dec) SPREAD1(nb, div, 2, true, b8); else SPREAD1(nb, div, 2, false, b8);                 \
    } else {                                                                                       \
      if (dec) SPREAD1(nb, div, 0, true, b8); else SPREAD1(nb, div, 0, false, b8);                 \
    }                                                                                              \
    return hipGetLastError();                                                                      \
  }
#if TD_PART == 1
SPREAD(TD_KIND_W16, 16, 0, false)
#elif TD_PART == 2
SPREAD(TD_KIND_W8, 8, 1, false)
#elif TD_PART == 3
SPREAD(TD_KIND_B16, 16, 1, true)
#elif TD_PART == 4
SPREAD(TD_KIND_B32, 32, 1, true)
#endif
#undef SPREAD
#undef SPREAD1

#define NO_ES (void)dg; (void)ng; (void)nblocks; (void)lds; (void)a; (void)es; (void)st; return hipErrorInvalidValue
#if TD_PART == 1
PART_FUNCS(TD_KIND_W16, BIDIR(16, 0, false), RUN1(16, 0, false), RUNES(16, 0, false))
#elif TD_PART == 2
PART_FUNCS(TD_KIND_W8, BIDIR(8, 1, false), RUN1(8, 1, false), RUNES(8, 1, false))
PART_FUNCS(TD_KIND_SSE, if (td_sched().sse_bidir) SEQT(k_sse_bidir, 128); else SEQ(k_sse_halfit), (void)n0; (void)nh; (void)lds; (void)dec; (void)a;
           return hipErrorInvalidValue,
           (void)lds; hipLaunchKernelGGL(k_sse_es<0>, dim3(nblocks), dim3(128), 0, st, dg, ng,
                                         (const s4 *)a.SP0, (s2 *)a.XP1, (s2 *)a.A, (uint32_t *)a.D,
                                         (const s2 *)a.T, a.plane, (s2 *)a.scratch, es))
PART_FUNCS(TD_KIND_GEN, SEQ(k_gen_halfit), (void)n0; (void)nh; (void)lds; (void)dec; (void)a;
           return hipErrorInvalidValue, NO_ES)
#elif TD_PART == 3
PART_FUNCS(TD_KIND_B16, BIDIR(16, 1, true), RUN1(16, 1, true), RUNES(16, 1, true))
#elif TD_PART == 4
PART_FUNCS(TD_KIND_B32, BIDIR(32, 1, true), RUN1(32, 1, true), RUNES(32, 1, true))
#endif
#undef NO_ES
#undef RUNES
#undef PART_FUNCS
#undef RUN1
#undef SEQ1
#undef SEQ
#undef SEQT
#undef BIDIR
#undef BIDIR1

#if TD_PART == 0
hipError_t launch_halfit(int n, int kind, const TdGroup *dg, int ng, int nblocks, size_t lds,
                         bool dec, const TdArrays &arr, const uint8_t *pair_done, hipStream_t st) {
  if (ng <= 0 || nblocks <= 0) return hipSuccess;
  const int mode = (n & 1) ? 1 : (n == 0 ? 2 : 0);
  TdArrays a = arr;
  if (!dec) a.D = nullptr;
  switch (kind) {
  case TD_KIND_W16: return halfit_part<TD_KIND_W16>(mode, dg, ng, nblocks, lds, dec, a, pair_done, st);
  case TD_KIND_W8: return halfit_part<TD_KIND_W8>(mode, dg, ng, nblocks, lds, dec, a, pair_done, st);
  case TD_KIND_SSE: return halfit_part<TD_KIND_SSE>(mode, dg, ng, nblocks, lds, dec, a, pair_done, st);
  case TD_KIND_GEN: return halfit_part<TD_KIND_GEN>(mode, dg, ng, nblocks, lds, dec, a, pair_done, st);
  case TD_KIND_B16: return halfit_part<TD_KIND_B16>(mode, dg, ng, nblocks, lds, dec, a, pair_done, st);
  case TD_KIND_B32: return halfit_part<TD_KIND_B32>(mode, dg, ng, nblocks, lds, dec, a, pair_done, st);
  default: return hipErrorInvalidValue;
  }
}

int spread_max_pairs() { return TD_SPREAD_MAX_PAIRS; }

bool spread_ok(int kind, int K, int nb) {
  const bool win = kind == TD_KIND_W16 || kind == TD_KIND_W8 || kind == TD_KIND_B16 || kind == TD_KIND_B32;
  return win && nb > 1 && K % nb == 0 && (K / nb) % TD_BIDIR_CW == 0 && K / nb >= 48;
}

hipError_t launch_halfit_spread(int n, int kind, const TdGroup *dg, int npairs, int K, int nb, bool dec,
                                const TdArrays &arr, const uint8_t *pair_done, hipStream_t st,
                                uint8_t *outb, size_t out_stride, const SpreadOut &so) {
  if (npairs <= 0) return hipSuccess;
  if (!spread_ok(kind, K, nb) || npairs > TD_SPREAD_MAX_PAIRS || K > 6144 ||
      K / TD_BIDIR_CW > TD_SPREAD_THREADS * TD_SPREAD_SPLIT || (outb && (!dec || !so.cnt)))
    return hipErrorInvalidValue;
  const int mode = (n & 1) ? 1 : (n == 0 ? 2 : 0);
  TdArrays a = arr;
  if (!dec) a.D = nullptr;
  const size_t lds = (size_t)(2 * (K / nb / TD_BIDIR_CW) + 1) * nb * 32;
  switch (kind) {
  case TD_KIND_W16: return spread_part<TD_KIND_W16>(mode, dg, npairs, lds, dec, a, pair_done, outb, out_stride, so, st);
  case TD_KIND_W8: return spread_part<TD_KIND_W8>(mode, dg, npairs, lds, dec, a, pair_done, outb, out_stride, so, st);
  case TD_KIND_B16: return spread_part<TD_KIND_B16>(mode, dg, npairs, lds, dec, a, pair_done, outb, out_stride, so, st);
  case TD_KIND_B32: return spread_part<TD_KIND_B32>(mode, dg, npairs, lds, dec, a, pair_done, outb, out_stride, so, st);
  default: return hipErrorInvalidValue;
  }
}

bool halfits_fusable(int kind) {
  return kind == TD_KIND_W16 || kind == TD_KIND_W8 || kind == TD_KIND_B16 || kind == TD_KIND_B32;
}

// early stop in one launch: the window kinds (k_win_bidir_es) and the two-wave SSE decoder (k_sse_es)
bool halfits_es_fusable(int kind) {
  if (kind == TD_KIND_SSE) return td_sched().sse_bidir != 0;
  return halfits_fusable(kind);
}

TdSched &td_sched() {
  static TdSched s = [] {
    auto env = [](const char *n, int d) {
      const char *e = getenv(n);
      return e && e[0] ? atoi(e) : d;
    };
    TdSched t{env("SRSGPU_TDEC_FUSED", 1) != 0, std::min(std::max(env("SRSGPU_ES_FUSED", 2), 0), 3),
              env("SRSGPU_ES_CHUNK", 8), env("SRSGPU_SSE_BIDIR", 1) != 0};
    if (t.es_chunk < 1) t.es_chunk = 1;
    return t;
  }();
  return s;
}

hipError_t launch_halfits(int n0, int nh, int kind, const TdGroup *dg, int ng, int nblocks,
                          size_t lds, bool dec, const TdArrays &a, hipStream_t st) {
  if (ng <= 0 || nblocks <= 0 || nh <= 0) return hipSuccess;
  switch (kind) {
  case TD_KIND_W16: return halfits_part<TD_KIND_W16>(n0, nh, dg, ng, nblocks, lds, dec, a, st);
  case TD_KIND_W8: return halfits_part<TD_KIND_W8>(n0, nh, dg, ng, nblocks, lds, dec, a, st);
  case TD_KIND_B16: return halfits_part<TD_KIND_B16>(n0, nh, dg, ng, nblocks, lds, dec, a, st);
  case TD_KIND_B32: return halfits_part<TD_KIND_B32>(n0, nh, dg, ng, nblocks, lds, dec, a, st);
  default: return hipErrorInvalidValue;
  }
}

hipError_t launch_halfits_es(int kind, const TdGroup *dg, int ng, int nblocks, size_t lds,
                             const TdArrays &a, const TdEs &es, hipStream_t st) {
  if (ng <= 0 || nblocks <= 0 || es.n1 <= es.n0) return hipSuccess;
  switch (kind) {
  case TD_KIND_SSE: return halfits_es_part<TD_KIND_SSE>(dg, ng, nblocks, lds, a, es, st);
  case TD_KIND_W16: return halfits_es_part<TD_KIND_W16>(dg, ng, nblocks, lds, a, es, st);
  case TD_KIND_W8: return halfits_es_part<TD_KIND_W8>(dg, ng, nblocks, lds, a, es, st);
  case TD_KIND_B16: return halfits_es_part<TD_KIND_B16>(dg, ng, nblocks, lds, a, es, st);
  case TD_KIND_B32: return halfits_es_part<TD_KIND_B32>(dg, ng, nblocks, lds, a, es, st);
  default: return hipErrorInvalidValue;
  }
}

hipError_t launch_pair_done(const TdGroup *dg, int ng, int npairs, const uint8_t *init_done, uint8_t *cb_done,
                            uint8_t *cb_ok, uint32_t *noi, uint8_t *pair_done, hipStream_t st,
                            uint32_t *run_cnt) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pair_done, dim3(nblk(npairs, 256)), dim3(256), 0, st, dg, ng, npairs, init_done,
                     cb_done, cb_ok, noi, pair_done, run_cnt);
  return hipGetLastError();
}

hipError_t launch_es_bytes(const TdGroup *dg, int ng, int npairs, const TdEs &es, hipStream_t st) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_es_bytes, dim3(nblk(npairs, ESB_PAIRS)), dim3(256), 0, st, dg, ng, npairs,
                     (const uint32_t *)es.dfz, es.outb, es.out_stride, es.cb_end,
                     knobs().tail_prio);
  return hipGetLastError();
}

hipError_t launch_decide(int n, const TdGroup *dg, int ng, int npairs, const TdArrays &a,
                         uint8_t *outb, size_t out_stride, bool early, uint8_t *cb_done,
                         uint8_t *cb_ok, uint32_t *noi, int max_halfits, uint8_t *pair_done,
                         hipStream_t st, uint32_t *run_list, uint32_t *run_cnt) {
  if (npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_decide, dim3(npairs), dim3(256), 0, st, n, dg, ng, (const uint32_t *)a.D, outb,
                     out_stride, early ? 1 : 0, cb_done, cb_ok, noi, max_halfits,
                     early ? pair_done : nullptr, knobs().decide_prio, early ? run_list : nullptr,
                     early ? run_cnt : nullptr, knobs().decide_words ? 1 : 0);
  return hipGetLastError();
}
#endif // TD_PART == 0

} // namespace srsgpu

#if defined(TD_TIMING) && TD_PART == 1
extern "C" int srsgpu_debug_td_chunk(unsigned long long *out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(srsgpu::td_chunk), sizeof(unsigned long long) * n) ==
                 hipSuccess
             ? 0
             : -1;
}
extern "C" int srsgpu_debug_td_times(unsigned long long *out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(srsgpu::td_times), sizeof(unsigned long long) * n) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
