"""Decoder scaling probe: time the fused fixed-iteration decoder (k_win_bidir_run, via
srsgpu_tdec_batch_run_dev) at 1024..4096 code blocks of K = 6144 with HIP-event timing of the
decoder kernel alone (srsgpu_prof). With one wave per SIMD at 4096 blocks, a purely issue-bound
kernel takes the same time per launch at fewer blocks (idle SIMDs), a purely traffic-bound one
scales with the blocks. Prints one line per size."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "empower-srslte_amd"))
import srsgpu_phy as s  # noqa: E402

K, NH = 6144, 8
stride = 3 * K + 12
rng = np.random.default_rng(0)
for N in (4096, 3072, 2048, 1024):
    b = s.TdecBatch(N, K, stream=torch.cuda.current_stream().cuda_stream)
    llr = torch.from_numpy(rng.integers(-60, 60, (N, stride)).astype(np.int16)).cuda()
    out = torch.zeros((N, K // 8), dtype=torch.uint8, device="cuda")
    for _ in range(20):
        assert b.run_dev(0, 0, llr.data_ptr(), stride, K, N, NH, out.data_ptr(), K // 8) == 0
    torch.cuda.synchronize()
    s.prof_reset()
    s.prof_enable(True)
    for _ in range(20):
        assert b.run_dev(0, 0, llr.data_ptr(), stride, K, N, NH, out.data_ptr(), K // 8) == 0
    torch.cuda.synchronize()
    s.prof_enable(False)
    ms, n = s.prof_get("k_win_bidir_run")
    per = ms / max(n, 1)
    print("N=%d: k_win_bidir_run %.1f us per launch, %.1f us per half-iteration, %.3f ns per CB-step"
          % (N, per * 1e3, per * 1e3 / NH, per * 1e6 / NH / (N * K) ), flush=True)
    b.close()
