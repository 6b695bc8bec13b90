"""Time one half-iteration-heavy decode for several batch sizes (GPU box).
Usage: python tools/sweep_batch.py [K] [halfits]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import srsgpu_phy as s  # noqa: E402
import torch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 6144
NH = int(sys.argv[2]) if len(sys.argv) > 2 else 8
stride = 3 * K + 12
maxn = 16384
rng = np.random.default_rng(0)
llr = torch.from_numpy(rng.integers(-300, 300, (maxn, stride), dtype=np.int16)).cuda()
out = torch.zeros((maxn, K // 8), dtype=torch.uint8, device="cuda")
b = s.TdecBatch(maxn, K, stream=torch.cuda.current_stream().cuda_stream)
for n in (256, 512, 1024, 2048, 4096, 8192, 16384):
    for _ in range(2):
        b.run_dev(0, 0, llr.data_ptr(), stride, K, n, NH, out.data_ptr(), K // 8)
    torch.cuda.synchronize()
    s.prof_reset()
    s.prof_enable(True)
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        b.run_dev(0, 0, llr.data_ptr(), stride, K, n, NH, out.data_ptr(), K // 8)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    s.prof_enable(False)
    km, kc = s.prof_get("halfit")
    print("n=%6d  step %.3f ms  %.2f Gbit/s  halfit avg %.1f us  per-CB-halfit %.3f us" %
          (n, dt * 1e3, n * K / dt / 1e9, km / kc * 1e3, km / kc * 1e3 / n), flush=True)
