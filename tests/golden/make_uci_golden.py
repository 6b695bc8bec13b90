"""Record golden UCI-on-PUSCH receptions from the reference build (`make -C oracle ref`): PUSCH TBs
with HARQ-ACK (1-2 bits), RI and CQI (block code up to 11 bits, convolutional code with CRC8 above)
multiplexed by srslte_ulsch_uci_encode (sch.c:994-1090), received as noisy int16 soft bits scrambled
by a PUSCH sequence, and decoded by the reference's srslte_pusch_decode steps (pusch.c:626-657:
srslte_ulsch_uci_decode_ri_ack, srslte_scrambling_s_offset, srslte_ulsch_uci_decode) through
oracle/ref_harness.c ref_ulsch_uci_decode. Recorded per case: the scrambled soft bits, the sequence,
the deinterleaved g bits, ACK / RI / cqi_ack / CQI bits, the return value and the decoded data.

    python tests/golden/make_uci_golden.py   -> tests/golden/uci_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import Oracle, PdschOracle, Ref, uci_case, uci_rx  # noqa: E402

# (tbs, Qm, nof_prb, nof_symb, O (ack, ri, cqi), I_off (ack, ri, cqi), M_sc_init_prb, sigma)
CASES = [
    (1544, 2, 10, 12, (1, 1, 0), (0, 2, 2), None, 25),
    (1544, 4, 10, 12, (2, 1, 0), (5, 5, 6), None, 25),
    (4008, 6, 20, 12, (2, 0, 11), (3, 0, 4), None, 25),
    (4008, 2, 20, 12, (1, 0, 30), (9, 0, 9), None, 10),
    (10296, 6, 50, 12, (1, 2, 7), (10, 6, 12), None, 25),
    (6200, 4, 25, 11, (2, 1, 4), (1, 1, 2), 30, 40),   # SRS symbol (11 columns), M_sc_init != M_sc
    (0, 2, 4, 12, (1, 1, 4), (0, 2, 2), None, 25),     # UCI without data (K = O_cqi)
    (0, 4, 6, 12, (0, 1, 64), (0, 4, 15), None, 5),
    (0, 2, 3, 12, (2, 0, 20), (14, 0, 15), None, 30),
    (25456, 6, 100, 12, (1, 1, 40), (12, 12, 15), None, 25),
]


def main():
    ref, orc = Ref(), Oracle()
    po = PdschOracle(orc)
    rng = np.random.default_rng(36212)
    arrays, man = {}, []
    for n, (tbs, Qm, prb, nsymb, O, I_off, msi, sigma) in enumerate(CASES):
        cqi = tuple(int(v) for v in rng.integers(0, 2, O[2]))
        ack = tuple(int(v) for v in rng.integers(0, 2, 2))
        u = uci_case(tbs, Qm, prb, nof_symb=nsymb, O=O, I_off=I_off, ack=ack, ri=int(rng.integers(0, 2)), cqi=cqi,
                     M_sc_init=12 * msi if msi else None)
        data = rng.integers(0, 256, tbs // 8 + 8).astype(np.uint8)
        qb = ref.uci_encode(u, data)
        c = po.sequence(int(rng.integers(1, 2 ** 30)), u["nof_bits"])
        qs = uci_rx(rng, qb, c, sigma=sigma)
        if tbs:
            ref.sb_reset(0)
        r, out, g, d, noi, crc = ref.uci_decode(0, u, qs, c)
        key = "u%d" % n
        arrays[key + "_q"], arrays[key + "_c"], arrays[key + "_g"] = qs, c, g
        arrays[key + "_out"] = out
        arrays[key + "_data"] = data[:tbs // 8]
        arrays[key + "_rx"] = d[:tbs // 8]
        u = dict(u, key=key, ret=int(r), noi=int(noi), cqi=list(cqi), ack=list(ack))
        man.append(u)
        print(key, "ret", r, "ack/ri/cqi_ack", list(out[:4]), "data", tbs == 0 or bool((d[:tbs // 8] == data[:tbs // 8]).all()))
    arrays["manifest"] = np.frombuffer(json.dumps(man).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "uci_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
