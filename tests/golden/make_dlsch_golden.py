"""Record golden DL-SCH vectors (rate matching + transport-block decode with HARQ) from the srsLTE
reference itself (sch.c / rm_turbo.c / softbuffer.c compiled by `make -C oracle ref`).

Each TB case is a HARQ sequence: the TB is encoded by the reference's own encoder
(srslte_dlsch_encode2, rv 0 first so the circular buffer is filled, sch.c:187-296), sent through
BPSK/AWGN per transmission (our own PRNG), quantised to int16 LLRs and decoded by
srslte_dlsch_decode2 into ONE persistent softbuffer until the TB passes. Stored per transmission:
the input LLRs and the reference's return code, data bytes ((tbs+24)/8), nof_iterations and
cb_crc flags. Also stored: de-rate-matching outputs (srslte_rm_turbo_rx_lut_) for a few (K, rv).

    python tests/golden/make_dlsch_golden.py   -> tests/golden/dlsch_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import DlschOracle, Oracle, Ref  # noqa: E402

# (tbs, Qm, nof_e_bits, snr_db list per transmission, rv order)
TB_CASES = [
    (75376, 6, 90000, [1.5, 3.0], [0, 2]),      # C3: 20 MHz MCS 28, 13 x K=5824
    (75376, 6, 90000, [6.0], [0]),              # error-free first transmission
    (31704, 6, 40008, [0.5, 1.0, 2.0], [0, 2, 3]),  # 6 CBs, HARQ combining
    (41536, 4, 60000, [3.0, 3.0], [0, 1]),      # C2 > 0 (K1 = 6016 / K2 = 5952 mix)
    (5736, 4, 12000, [2.0, 3.0], [0, 2]),       # C = 1, K = 5760: CRC24A over tbs+24
    (1000, 2, 3000, [-1.0, 0.5, 2.0], [0, 2, 3, 1]),  # C = 1, SSE16 window (K = 1024? no: AVX)
    (376, 2, 1200, [1.0, 2.0], [0, 3]),         # K = 400: SSE non-window, natural table
    (16, 2, 200, [2.0], [0]),                   # K = 40
    (6136, 6, 9000, [2.5, 3.5], [0, 2]),        # C = 2 (K1 = 3136? filled by cbsegm)
    (1608, 4, 1500, [6.0, 6.0], [0, 2]),        # punctured (E < K): may need the retransmission
]
RM_CASES = [(40, 0, 0), (512, 1, 1), (800, 2, 1), (1056, 3, 1), (5824, 0, 1), (6144, 2, 0)]


def main():
    o, r = Oracle(), Ref()
    d = DlschOracle(o)
    rng = np.random.default_rng(20181009)
    arrays, manifest = {}, []
    for ci, (tbs, Qm, nb, snrs, rvs) in enumerate(TB_CASES):
        seg = o.cbsegm(tbs)
        assert seg[5] == 0, ("filler bits", tbs)
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        key = "tb%02d" % ci
        arrays[key + "_data"] = data
        r.sb_reset(0)
        steps = []
        for t, rv in enumerate(rvs):
            snr = snrs[min(t, len(snrs) - 1)]
            e = r.encode(tbs, rv, Qm, nb, data)
            assert (e == d.encode(tbs, rv, Qm, nb, data)).all(), ("encoder drift", key, rv)
            sigma = np.float32(10 ** (-snr / 20))
            y = np.where(e == 1, np.float32(1), np.float32(-1)) + sigma * rng.standard_normal(
                e.size).astype(np.float32)
            llr = (np.float32(100) * y).astype(np.int16)
            ret, dout, noi, cb_crc = r.decode(0, tbs, rv, Qm, llr, 8)
            sk = "%s_t%d" % (key, t)
            arrays[sk + "_llr"] = llr
            arrays[sk + "_out"] = dout[:(tbs + 24) // 8]
            arrays[sk + "_cbcrc"] = cb_crc
            steps.append(dict(rv=rv, snr=snr, ret=int(ret), noi=int(noi)))
            if ret == 0:
                break
        manifest.append(dict(key=key, kind="tb", tbs=tbs, Qm=Qm, nbits=nb, C=seg[0], steps=steps,
                             max_halfits=8))
    for ci, (K, rv, sb) in enumerate(RM_CASES):
        N = 3 * K + 12
        e = rng.integers(-20000, 20000, int(N * 1.7)).astype(np.int16)
        out = np.zeros(3 * (K + 32) + 12, np.int16)
        r.rm_rx(e, out, K, rv, sb)
        key = "rm%02d" % ci
        arrays[key + "_in"] = e
        arrays[key + "_out"] = out
        manifest.append(dict(key=key, kind="rm", K=K, rv=rv, sb=sb))
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "dlsch_golden.npz"), **arrays)
    print(json.dumps(manifest, indent=0)[:3000])


if __name__ == "__main__":
    main()
