// Wave issue priority for latency-critical launches that run beside other streams' throughput
// kernels: s_setprio raises the wave's priority in its SIMD's instruction arbitration (0 = default).
// Plus the process-wide tuning knobs those launches read: a snapshot of the environment taken once
// (first use) and replaced only by srsgpu_knobs_reload(), so no launch calls getenv (a getenv on a
// queue's dispatcher thread racing a setenv elsewhere is undefined behaviour in glibc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <atomic>

namespace srsgpu {
__device__ __forceinline__ void wave_prio(int prio) {
  switch (__builtin_amdgcn_readfirstlane(prio)) {
  case 1: __builtin_amdgcn_s_setprio(1); break;
  case 2: __builtin_amdgcn_s_setprio(2); break;
  case 3: __builtin_amdgcn_s_setprio(3); break;
  default: break;
  }
}

struct Knobs {
  int es_prio;     // SRSGPU_ES_PRIO (0..3, default 3): the early-stop decoder launches
  int tail_prio;   // SRSGPU_TAIL_PRIO (default 3): k_es_bytes, k_tb_finish
  int decide_prio; // SRSGPU_DECIDE_PRIO (default: tail_prio): k_decide
  int h0_prio;     // SRSGPU_H0_PRIO (default 0): the first half-iteration
  bool llr_generic; // SRSGPU_LLR_GENERIC (A/B): the general PDSCH LLR kernel only
  bool llr_noxcd;   // SRSGPU_LLR_NOXCD (A/B): the plain item-major workgroup mapping
  bool es_compact;  // SRSGPU_ES_COMPACT (default 1): the hybrid early-stop launch packs the running pairs
  bool defer_p1;    // SRSGPU_DEFER_P1 (default 1): k_load_derm leaves P1 to the pairs still running
  bool h0_decide;   // SRSGPU_H0_DECIDE=1 (A/B, default 0): the hybrid schedule's first half-iteration
                    // checks its own blocks (k_win_bidir_h0c: bytes written at once), no k_decide launch;
                    // slower (r06_s10: 0.799 against 0.770 ms per batch: the check lengthens every
                    // decoder workgroup's life on its CU, where k_decide's 3,328 small ones overlap)
  bool ldderm_fast; // SRSGPU_LDERM_FAST (default 1): k_load_derm's branch-free form for fresh, staged,
                    // same-table 16-bit pairs
  bool decide_words; // SRSGPU_DECIDE_WORDS (default 1): k_decide writes DEC1 bytes as 32-bit words
  bool split_early;  // SRSGPU_SPLIT_EARLY (default 1): a tail stream takes over right after the first
                     // half-iteration (r06_s14, one lane: 0.721 against 0.764 ms per batch)
  bool spread;       // SRSGPU_SPREAD (default 1): per-half-iteration launches of a few pairs run as
                     // k_win_spread (one pair per workgroup, both recursions whole, then every chunk
                     // in parallel): the drop-in srslte_tdec_iteration's latency
  bool spread_poll;  // SRSGPU_SPREAD_POLL (default 1): the drop-in waits for k_win_spread's host-mapped
                     // completion word instead of synchronising the stream
};

inline int env_prio(const char *name, int dflt) {
  const char *e = getenv(name);
  if (!e || !e[0]) return dflt;
  const int v = atoi(e);
  return v < 0 ? 0 : (v > 3 ? 3 : v);
}

inline const Knobs *knobs_from_env() {
  Knobs *k = new Knobs;
  k->es_prio = env_prio("SRSGPU_ES_PRIO", 3);
  k->tail_prio = env_prio("SRSGPU_TAIL_PRIO", 3);
  k->decide_prio = env_prio("SRSGPU_DECIDE_PRIO", k->tail_prio);
  k->h0_prio = env_prio("SRSGPU_H0_PRIO", 0);
  k->llr_generic = getenv("SRSGPU_LLR_GENERIC") != nullptr;
  k->llr_noxcd = getenv("SRSGPU_LLR_NOXCD") != nullptr;
  {
    const char *e = getenv("SRSGPU_ES_COMPACT");
    k->es_compact = !(e && e[0] == '0');
    const char *f = getenv("SRSGPU_DEFER_P1");
    k->defer_p1 = !(f && f[0] == '0');
    const char *h = getenv("SRSGPU_H0_DECIDE");
    k->h0_decide = h && h[0] == '1';
    const char *l = getenv("SRSGPU_LDERM_FAST");
    k->ldderm_fast = !(l && l[0] == '0');
    const char *w = getenv("SRSGPU_DECIDE_WORDS");
    k->decide_words = !(w && w[0] == '0');
    const char *se = getenv("SRSGPU_SPLIT_EARLY");
    k->split_early = !(se && se[0] == '0');
    const char *sp = getenv("SRSGPU_SPREAD");
    k->spread = !(sp && sp[0] == '0');
    const char *spp = getenv("SRSGPU_SPREAD_POLL");
    k->spread_poll = !(spp && spp[0] == '0');
  }
  return k;
}

inline std::atomic<const Knobs *> &knobs_slot() {
  static std::atomic<const Knobs *> p{nullptr};
  return p;
}

// the current snapshot (a replaced one is never freed: a launch on another thread may still read it)
inline const Knobs &knobs() {
  const Knobs *k = knobs_slot().load(std::memory_order_acquire);
  if (k) return *k;
  const Knobs *n = knobs_from_env();
  if (knobs_slot().compare_exchange_strong(k, n, std::memory_order_acq_rel)) return *n;
  delete n;
  return *k;
}
} // namespace srsgpu
