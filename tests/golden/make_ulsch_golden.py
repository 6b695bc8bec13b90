"""Record golden UL-SCH vectors from the srsLTE reference itself (sch.c compiled by
`make -C oracle ref`): srslte_ulsch_encode (sch.c:987-1090, no UCI: encode_tb_off + the 36.212
5.2.2.8 channel interleaver) makes the q bits of a PUSCH transport block, BPSK/AWGN per
transmission (our own PRNG) gives int16 LLRs, and srslte_ulsch_decode (sch.c:883-889: channel
deinterleaver + decode_tb) decodes them into ONE persistent softbuffer over a HARQ sequence until
the TB passes. Stored per transmission: the q-bit LLRs and the reference's return code, data bytes
((tbs+24)/8), nof_iterations and cb_crc flags.

    python tests/golden/make_ulsch_golden.py   -> tests/golden/ulsch_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import DlschOracle, Oracle, Ref  # noqa: E402

# (tbs, Qm, nof_prb, nof_symb, snr_db per transmission, rv order); nof_bits = 12 nof_prb nof_symb Qm
# (nof_symb 12: normal CP, 11: an SRS symbol shortened)
TB_CASES = [
    (600, 2, 6, 12, [2.0], [0]),                  # C = 1, small
    (1544, 2, 6, 12, [-1.0, 1.0, 3.0], [0, 2, 3]),  # C = 1 at a high code rate: HARQ needed
    (4008, 2, 25, 11, [1.0, 2.0], [0, 2]),        # SRS-shortened subframe
    (8760, 4, 25, 12, [3.0, 5.0], [0, 2]),        # C = 2, 16QAM columns of 4
    (30576, 6, 50, 12, [3.0, 4.0, 6.0], [0, 2, 3, 1]),  # 64QAM, 5 CBs
    (40576, 4, 100, 12, [2.0, 4.0], [0, 2]),      # 100 PRB, 7 CBs
    (51024, 6, 100, 11, [5.0, 6.0], [0, 2]),      # 64QAM with SRS
    (75376, 6, 100, 12, [8.0], [0]),              # error-free first transmission, 13 CBs
]


def main():
    o, r = Oracle(), Ref()
    d = DlschOracle(o)
    rng = np.random.default_rng(20181017)
    arrays, manifest = {}, []
    for ci, (tbs, Qm, prb, ns, snrs, rvs) in enumerate(TB_CASES):
        seg = o.cbsegm(tbs)
        assert seg[5] == 0, ("filler bits", tbs)
        nb = 12 * prb * ns * Qm
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        key = "ul%02d" % ci
        arrays[key + "_data"] = data
        r.sb_reset(0)
        steps = []
        for t, rv in enumerate(rvs):
            snr = snrs[min(t, len(snrs) - 1)]
            q = r.ul_encode(tbs, rv, Qm, nb, ns, data)
            sigma = np.float32(10 ** (-snr / 20))
            y = np.where(q == 1, np.float32(1), np.float32(-1)) + sigma * rng.standard_normal(
                q.size).astype(np.float32)
            llr = (np.float32(100) * y).astype(np.int16)
            ret, dout, noi, cb_crc = r.ul_decode(0, tbs, rv, Qm, ns, llr, 8)
            sk = "%s_t%d" % (key, t)
            arrays[sk + "_llr"] = llr
            arrays[sk + "_out"] = dout[:(tbs + 24) // 8]
            arrays[sk + "_cbcrc"] = cb_crc
            steps.append(dict(rv=rv, snr=snr, ret=int(ret), noi=int(noi)))
            if ret == 0:
                break
        manifest.append(dict(key=key, tbs=tbs, Qm=Qm, nof_prb=prb, nof_symb=ns, nbits=nb, C=seg[0],
                             steps=steps, max_halfits=8))
        print(key, tbs, Qm, prb, ns, seg[0], steps)
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "ulsch_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
