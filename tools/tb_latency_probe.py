"""Per-call latency of the whole-TB drop-in level: ONE transport block per srsgpu_dlsch_decode call
(what srslte_dlsch_decode2 in integration/srslte_gpu_shim.c does per call, sch.c:500-512) against the
reference's srslte_dlsch_decode2 on one CPU core (oracle/_ref, compiled from the reference's sources)
on the same LLRs: TBS 75,376 (13 code blocks), 64QAM, 90,000 coded bits, at two SNRs. Host
pointers in and out, as the drop-in sees them; the outputs are checked equal. argv[1]: output JSON."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import srsgpu_phy as s  # noqa: E402
from srsgpu_testlib import Ref  # noqa: E402

ref = Ref()
TBS, QM, NB, NTB = 75376, 6, 90000, 24
rng = np.random.default_rng(11)
g = s.Dlsch(1, 16, 64)
res = {"tbs": TBS, "Qm": QM, "nof_e_bits": NB, "transport_blocks": NTB, "points": []}
for snr in (20.0, 6.0):
    cases = []
    for i in range(NTB):
        data = rng.integers(0, 256, TBS // 8).astype(np.uint8)
        e = ref.encode(TBS, 0, QM, NB, data)
        y = np.where(e == 1, 1.0, -1.0) + 10 ** (-snr / 20) * rng.standard_normal(e.size)
        cases.append((100 * y).astype(np.float32).astype(np.int16))
    tb = dict(tbs=TBS, rv=0, Qm=QM, nof_e_bits=NB, softbuffer=0)
    for llr in cases[:3]:  # warm-up
        g.reset(0)
        g.decode([tb], [llr], 8)
    tg, tc, same, nois = [], [], 0, []
    for llr in cases:
        g.reset(0)
        t0 = time.perf_counter()
        ret, data, noi = g.decode([tb], [llr], 8)
        tg.append(time.perf_counter() - t0)
        ref.sb_reset(0)
        t0 = time.perf_counter()
        r, od, onoi, _ = ref.decode(0, TBS, 0, QM, llr, 8)
        tc.append(time.perf_counter() - t0)
        nb = (TBS + 24) // 8
        same += int(ret[0] == r and noi[0] == onoi and (data[0][:nb] == od[:nb]).all())
        nois.append(int(noi[0]))
    res["points"].append({"snr_db": snr, "gpu_us_per_tb_median": round(1e6 * float(np.median(tg)), 1),
                          "cpu_ref_us_per_tb_one_core_median": round(1e6 * float(np.median(tc)), 1),
                          "equal_outputs": "%d/%d" % (same, NTB), "noi_mean": round(float(np.mean(nois)), 2)})
g.close()
print(json.dumps(res))
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
