/*
 * Multi-GPU work partitioning for the batched receive path.
 *
 * Code blocks, transport blocks and subframes are independent: the math has no exchange step, so a
 * job is split across ranks (one process per GPU) with no data-path collective. The reference has
 * no device split at all; its only parallel analogues are the PHY worker pool, which hands whole
 * subframes to idle workers (srsue/src/phy/phy.cc:141-168), and the PDSCH coworker thread that
 * decodes TB0 beside TB1 (lib/src/phy/phch/pdsch.c:949-999). These functions are the multi-GPU
 * counterpart of that hand-out, host-only, and deterministic: every rank computes the same
 * partition from the same inputs, so no rank needs to be told what the others hold.
 */
#ifndef SRSGPU_SHARD_H
#define SRSGPU_SHARD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Contiguous ranges (C2-C4: code-block / subframe batches of equal cost): rank r of world owns
 * units [first[r], first[r + 1]); first has world + 1 entries, first[0] = 0, first[world] = n.
 * Range sizes differ by at most one. Returns 0, or -1 on invalid arguments. */
int srsgpu_shard_contiguous(uint32_t n, uint32_t world, uint32_t *first);

/* Weighted binning from one global queue (C5: mixed-size transport blocks): units are taken in
 * decreasing weight (ties: lower index first) and each goes to the rank with the smallest load so
 * far (ties: lower rank) — longest-processing-time-first list scheduling, whose makespan is within
 * 4/3 of the optimum. weight[i] is the unit's decoding cost, e.g. sum of K over its code blocks
 * times the half-iteration budget. owner[i] receives the rank of unit i; load (world entries, may
 * be NULL) the summed weight per rank. Returns 0, or -1 on invalid arguments. */
int srsgpu_shard_weighted(const uint64_t *weight, uint32_t n, uint32_t world, int32_t *owner,
                          uint64_t *load);

#ifdef __cplusplus
}
#endif
#endif
