"""Time one 4096 x K=6144, 8-half-iteration decode with a given build of the library (experiments:
python3 tools/dec_time.py empower-srslte_amd/lib/exp/libsrsgpu_phy.so). Prints ms per batch."""
import ctypes
import sys

import numpy as np
import torch

lib = ctypes.CDLL(sys.argv[1])
vp = ctypes.c_void_p
K, N, NH = 6144, 4096, 8
q = vp()
assert lib.srsgpu_tdec_batch_create(ctypes.byref(q), N, K) == 0
stride = 3 * K + 12
rng = np.random.default_rng(0)
llr = torch.from_numpy(rng.integers(-60, 60, (N, stride)).astype(np.int16)).cuda()
out = torch.zeros((N, K // 8), dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
lib.srsgpu_tdec_batch_set_stream(q, vp(s.cuda_stream))
def run():
    assert lib.srsgpu_tdec_batch_run_dev(q, 0, 0, vp(llr.data_ptr()), ctypes.c_size_t(stride), K, N, NH,
                                         vp(out.data_ptr()), ctypes.c_size_t(K // 8)) == 0
torch.cuda.synchronize()
for _ in range(40):
    run()
s.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
with torch.cuda.stream(s):
    e0.record()
    for _ in range(20):
        run()
    e1.record()
s.synchronize()
print("%s: %.1f us per batch" % (sys.argv[1], e0.elapsed_time(e1) * 1e3 / 20))
