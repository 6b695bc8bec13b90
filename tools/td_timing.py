"""Phase timing of the bidirectional decoder kernel (debug build: make -C empower-srslte_amd timing).

Loads lib/timing/libsrsgpu_phy.so directly (not the product library), runs one 4096 x K=6144
batch with 8 half-iterations and prints, per phase, the mean shader-clock cycles over waves of
the last launch: prepass, first half (recursion + checkpoints), barrier wait, second half (LLRs).
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(REPO, "empower-srslte_amd", "lib", "timing", "libsrsgpu_phy.so"))
vp = ctypes.c_void_p
K, N, NH = 6144, int(sys.argv[1]) if len(sys.argv) > 1 else 4096, 8
q = vp()
assert lib.srsgpu_tdec_batch_create(ctypes.byref(q), N, K) == 0
stride = 3 * K + 12
rng = np.random.default_rng(0)
llr = torch.from_numpy(rng.integers(-60, 60, (N, stride)).astype(np.int16)).cuda()
out = torch.zeros((N, K // 8), dtype=torch.uint8, device="cuda")
lib.srsgpu_tdec_batch_set_stream(q, vp(torch.cuda.current_stream().cuda_stream))
for _ in range(3):
    assert lib.srsgpu_tdec_batch_run_dev(q, 0, 0, vp(llr.data_ptr()), ctypes.c_size_t(stride), K, N, NH,
                                         vp(out.data_ptr()), ctypes.c_size_t(K // 8)) == 0
torch.cuda.synchronize()
nw = min(N // 4, 2048)  # waves: 2 per block of 64 chains (4 pairs), blocks < 1024 stamped
t = (ctypes.c_ulonglong * (2048 * 8))()
assert lib.srsgpu_debug_td_times(t, 2048 * 8) == 0
a = np.frombuffer(t, dtype=np.uint64).reshape(2048, 8)[:nw].astype(np.int64)
names = ["prepass", "first half", "barrier wait", "second half"]
for role in (0, 1):
    r = a[role::2]
    d = np.diff(r[:, :5], axis=1)
    print("wave %d (%s):" % (role, "alpha" if role == 0 else "beta"),
          ", ".join("%s %.0f" % (n, v) for n, v in zip(names, d.mean(0))), "total %.0f" % (r[:, 4] - r[:, 0]).mean())
wall = (a[:, 6] - a[:, 5]).astype(np.float64) / 100e6  # wall_clock64: 100 MHz
clk = (a[:, 4] - a[:, 0]).astype(np.float64)
print("per-wave wall %.1f us (mean), shader clock %.2f GHz (mean), kernel span %.1f us" %
      (wall.mean() * 1e6, (clk / wall).mean() / 1e9, (a[:, 6].max() - a[:, 5].min()) / 100.0))
st = (a[:, 5] - a[:, 5].min()).astype(np.float64) / 100.0  # us
en = (a[:, 6] - a[:, 5].min()).astype(np.float64) / 100.0
valid = st < 1e4
print("wave start times (us from first): percentiles 0/25/50/75/100:",
      np.percentile(st[valid], [0, 25, 50, 75, 100]).round(1), " ends:", np.percentile(en[valid], [0, 50, 100]).round(1),
      " valid", valid.sum())
hist, edges = np.histogram(st[valid], bins=10)
print("start histogram:", hist.tolist(), edges.round(1).tolist())
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
assert lib.srsgpu_tdec_batch_run_dev(q, 0, 0, vp(llr.data_ptr()), ctypes.c_size_t(stride), K, N, NH,
                                     vp(out.data_ptr()), ctypes.c_size_t(K // 8)) == 0
ev1.record()
torch.cuda.synchronize()
print("one batch (load + %d half-its + decide): %.1f us" % (NH, ev0.elapsed_time(ev1) * 1e3))

# per-chunk stamps (td_chunk): phase-1 chunk starts, phase-2 chunk start / betas done / LLRs done
c = (ctypes.c_ulonglong * (2048 * 80))()
if hasattr(lib, "srsgpu_debug_td_chunk") and lib.srsgpu_debug_td_chunk(c, 2048 * 80) == 0:
    ch = np.frombuffer(c, dtype=np.uint64).reshape(2048, 80)[:nw].astype(np.int64)
    for role in (0, 1):
        r = ch[role::2]
        t0 = a[role::2, 0]
        p1 = r[:, :12] - t0[:, None]
        print("wave %d phase-1 chunk starts (cycles from wave start):" % role, p1.mean(0).round(0).tolist())
        p2 = r[:, 32:32 + 36].reshape(-1, 12, 3)
        betas = (p2[:, :, 1] - p2[:, :, 0]).mean(0)
        llrs = (p2[:, :, 2] - p2[:, :, 1]).mean(0)
        gaps = (p2[:, 1:, 0] - p2[:, :-1, 2]).mean(0)
        print("wave %d phase-2 betas per chunk:" % role, betas.round(0).tolist())
        print("wave %d phase-2 LLRs per chunk: " % role, llrs.round(0).tolist())
        print("wave %d phase-2 gaps between chunks:" % role, gaps.round(0).tolist())
