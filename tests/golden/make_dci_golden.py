"""Record golden DCI-candidate decodes from the reference build (`make -C oracle ref`): the
reference's srslte_rm_conv_rx, srslte_viterbi_decode_f and CRC16 composed as
srslte_pdcch_decode_msg / srslte_pdcch_dci_decode call them (pdcch.c:322-396), on random LLRs of
the PDCCH formats' lengths E = 72 L (L = 1, 2, 4, 8) and DCI sizes of 1.4-20 MHz cells, amplitudes
from below the decode threshold (mean |llr| <= 0.5: skipped) to clean.

    python tests/golden/make_dci_golden.py   -> tests/golden/dci_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import Ref, dci_decode  # noqa: E402


def main():
    ref = Ref()
    rng = np.random.default_rng(1906)
    arrays, manifest = {}, []
    for E in (72, 144, 288, 576):
        for nb in (19, 21, 25, 27, 31, 43, 57):
            for amp in (0.25, 0.7, 2.0):
                key = "d_%d_%d_%g" % (E, nb, amp)
                e = (amp * (rng.standard_normal(E) + np.where(rng.random(E) < 0.5, 1, -1))).astype(np.float32)
                r, d, c = dci_decode(ref, e, nb, ref=True)
                arrays[key + "_e"] = e
                arrays[key + "_bits"] = d
                manifest.append({"key": key, "E": E, "nof_bits": nb, "decoded": r, "crc_rem": c})
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "dci_golden.npz"), **arrays)
    print("wrote", len(manifest), "cases")


if __name__ == "__main__":
    main()
