// Multi-GPU partitioning of a receive job (include/srsgpu/shard.h). Host-only:
// the partition is computed identically on every rank, so the split itself needs no collective.
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <functional>
#include <numeric>
#include <queue>
#include <utility>
#include <vector>

#include "srsgpu/shard.h"

extern "C" {

int srsgpu_shard_contiguous(uint32_t n, uint32_t world, uint32_t *first) {
  if (world == 0 || !first) return -1;
  for (uint32_t r = 0; r <= world; r++) first[r] = (uint32_t)(((uint64_t)n * r) / world);
  return 0;
}

int srsgpu_shard_weighted(const uint64_t *weight, uint32_t n, uint32_t world, int32_t *owner,
                          uint64_t *load) {
  if (world == 0 || (n && (!weight || !owner))) return -1;
  std::vector<uint32_t> order(n);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return weight[a] > weight[b]; });
  // min-heap of (load, rank): the least loaded rank, lowest rank on ties
  typedef std::pair<uint64_t, uint32_t> Slot;
  std::priority_queue<Slot, std::vector<Slot>, std::greater<Slot>> heap;
  for (uint32_t r = 0; r < world; r++) heap.push(Slot(0, r));
  for (uint32_t i : order) {
    Slot s = heap.top();
    heap.pop();
    owner[i] = (int32_t)s.second;
    s.first += weight[i];
    heap.push(s);
  }
  if (load) {
    std::fill(load, load + world, 0);
    while (!heap.empty()) {
      load[heap.top().second] = heap.top().first;
      heap.pop();
    }
  }
  return 0;
}

} // extern "C"
