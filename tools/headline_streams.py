"""Headline decoder batches (4096 x K6144, 8 half-its) issued on 1 or 2 alternating streams."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
import torch  # noqa: E402
import srsgpu_phy as s  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
K, NCB, NH = 6144, 4096, 8
tcod = s.Tcod(K)
bits, idx, llr = bench.make_inputs(NCB, 1234, tcod)
d_in = torch.from_numpy(llr).to(dev)
stride = 3 * K + 12
for ns in (1, 2, 3, 4, 1, 3, 2):
    sts = [torch.cuda.Stream(dev) for _ in range(ns)]
    bs = [s.TdecBatch(NCB, K, stream=st.cuda_stream) for st in sts]
    outs = [torch.zeros((NCB, K // 8), dtype=torch.uint8, device=dev) for _ in range(ns)]

    def step(i):
        j = i % ns
        assert bs[j].run_dev(0, 0, d_in.data_ptr(), stride, K, NCB, NH, outs[j].data_ptr(), K // 8) == 0

    for i in range(4):
        step(i)
    torch.cuda.synchronize()
    n = 60
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(ns, "streams: %.3f ms/batch, %.1f Gbit/s" % (el / n * 1e3, NCB * K * n / el / 1e9), flush=True)
    for b in bs:
        b.close()
