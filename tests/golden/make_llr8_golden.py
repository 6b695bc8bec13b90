"""Record golden vectors of the reference's 8-bit LLR receive chain (llr_is_8bit: pdsch.c:795-806,
sch.c:344-364) from the srsLTE reference itself (demod_soft.c, scrambling.c, rm_turbo.c, sch.c,
turbodecoder*.c compiled by `make -C oracle ref`):

- srslte_demod_soft_demodulate_b for QPSK / 16QAM / 64QAM, symbol counts around the 8-symbol
  SIMD blocks (body and C tail) and amplitudes that saturate;
- srslte_scrambling_sb_offset with the PDSCH sequence;
- srslte_rm_turbo_rx_lut_8bit (int8 wrapping accumulation, the 8-bit decoder's sub-block table)
  for a few (K, rv, length), on top of a non-zero row;
- srslte_dlsch_decode2 with llr_is_8bit over HARQ sequences on one persistent softbuffer: the TB
  encoded by our oracle encoder (bit-exact with srslte_dlsch_encode2, tests/test_dlsch_oracle.py),
  BPSK/AWGN per transmission with our own PRNG, int8 LLRs; stored per transmission: input LLRs,
  return code, data bytes, nof_iterations, cb_crc.

    python tests/golden/make_llr8_golden.py   -> tests/golden/llr8_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import DlschOracle, Llr8, Oracle, Ref  # noqa: E402

DEMOD_N = [1, 7, 8, 9, 16, 23, 100, 1203]
DEMOD_AMP = [0.5, 1.0, 4.0]
# (K, rv, E): E below, at and above the circular buffer (wrap-around)
RM_CASES = [(40, 0, 100), (512, 1, 1548), (1056, 3, 4000), (2112, 2, 6348), (5824, 0, 9000),
            (6144, 2, 40000)]
# (tbs, Qm, nof_e_bits, amplitude, sigma per transmission, rv order): 8-bit HARQ combining wraps
# at 8 bits, so the amplitude is kept small
TB_CASES = [
    (1544, 2, 3000, 10, [1.3, 1.3, 1.1, 0.8], [0, 2, 3, 1]),
    (6712, 4, 7200, 10, [1.3, 1.3, 1.1, 0.8], [0, 2, 3, 1]),
    (20616, 6, 21000, 10, [1.3, 1.3, 1.1, 0.8], [0, 2, 3, 1]),
    (75376, 6, 84000, 10, [1.0, 0.9], [0, 2]),      # C3's TB: 13 x K = 5824 (AVX8 window)
    (75376, 6, 84000, 12, [0.3], [0]),
    (2280, 2, 8000, 10, [1.3, 1.3], [0, 2]),
    (31704, 4, 40000, 10, [1.3, 1.3, 1.1, 0.8], [0, 2, 3, 1]),
    (120, 2, 600, 10, [1.3, 1.0], [0, 2]),          # K = 144: 16-bit SSE fallback, natural rows
    (4008, 2, 6000, 10, [1.3, 1.3, 1.1], [0, 2, 3]),
]


def main():
    orc, ref = Oracle(), Ref()
    r = Llr8(ref, ref=True)
    dl = DlschOracle(orc)
    rng = np.random.default_rng(20261017)
    arrays, manifest = {}, []
    for mod in (1, 2, 3):
        for n in DEMOD_N:
            for amp in DEMOD_AMP:
                key = "demod_%d_%d_%g" % (mod, n, amp)
                sym = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * amp).astype(np.complex64)
                arrays[key + "_sym"] = sym
                arrays[key + "_llr"] = r.demod(mod, sym)
                manifest.append({"kind": "demod", "key": key, "mod": mod})
    for n, (rnti, q, nslot, cell) in zip([1, 33, 1000, 5001], [(1234, 0, 2, 1), (61, 1, 7, 300),
                                                               (65535, 0, 19, 503), (1, 1, 0, 0)]):
        key = "scr_%d" % n
        llr = rng.integers(-128, 128, n).astype(np.int8)
        arrays[key + "_in"] = llr
        arrays[key + "_out"] = r.scramble(rnti, q, nslot, cell, llr)
        manifest.append({"kind": "scramble", "key": key, "rnti": rnti, "q": q, "nslot": nslot,
                         "cell_id": cell})
    for K, rv, E in RM_CASES:
        key = "rm_%d_%d_%d" % (K, rv, E)
        e = rng.integers(-128, 128, E).astype(np.int8)
        init = rng.integers(-128, 128, 3 * (K + 32) + 12).astype(np.int8)
        out = np.zeros(18600 * 2, np.int8)
        out[:init.size] = init
        r.rm_rx(e, out, K, rv)
        arrays[key + "_e"] = e
        arrays[key + "_init"] = init
        arrays[key + "_out"] = out[:init.size]
        manifest.append({"kind": "rm", "key": key, "K": K, "rv": rv})
    for ci, (tbs, Qm, nbits, amp, sigmas, rvs) in enumerate(TB_CASES):
        data = rng.integers(0, 256, tbs // 8).astype(np.uint8)
        ref.sb_reset(0)
        tx = []
        for t, (sig, rv) in enumerate(zip(sigmas, rvs)):
            bits = dl.encode(tbs, rv, Qm, nbits, data)
            llr = np.clip(np.rint(amp * (np.where(bits == 1, 1.0, -1.0)
                                         + sig * rng.standard_normal(nbits))), -128, 127).astype(np.int8)
            ret, out, noi, crc = r.decode(0, tbs, rv, Qm, llr, 8)
            key = "tb%d_%d" % (ci, t)
            arrays[key + "_llr"] = llr
            arrays[key + "_data"] = out[:(tbs + 24) // 8]
            arrays[key + "_cbcrc"] = crc.astype(np.uint8)
            tx.append({"key": key, "rv": rv, "ret": int(ret), "noi": int(noi)})
        arrays["tb%d_tx" % ci] = data
        manifest.append({"kind": "tb", "key": "tb%d" % ci, "tbs": tbs, "Qm": Qm, "nbits": nbits,
                         "tx": tx})
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "llr8_golden.npz"), **arrays)
    print("wrote", len(manifest), "cases")


if __name__ == "__main__":
    main()
