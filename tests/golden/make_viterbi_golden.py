"""Record golden PDCCH Viterbi vectors from the reference build (`make -C oracle ref`):
srslte_viterbi_decode_f on the tail-biting K=7 r=1/3 decoder pdcch.c builds (:79), which on an AVX2
build is the 16-bit decoder (viterbi.c VITERBI_16). Frame lengths of the DCI formats + 16 CRC bits
and beyond, random +-1 code symbols with Gaussian noise from high to very low SNR, and a frame
scaled to tiny amplitudes (the quantiser's gain 1000 / max|x|).

    python tests/golden/make_viterbi_golden.py   -> tests/golden/viterbi_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import Ref, viterbi_tb_decode_f  # noqa: E402


def main():
    ref = Ref()
    rng = np.random.default_rng(37)
    arrays, manifest = {}, []
    for F in (24, 37, 41, 43, 47, 57, 58, 73, 100, 192):
        for snr in (-3.0, 0.0, 3.0, 20.0):
            key = "v_%d_%g" % (F, snr)
            x = (rng.standard_normal(3 * F) + 10 ** (snr / 20) * np.where(rng.random(3 * F) < 0.5, 1, -1))
            x = x.astype(np.float32)
            if F == 43:
                x = (x * 1e-4).astype(np.float32)
            arrays[key + "_sym"] = x
            arrays[key + "_out"] = viterbi_tb_decode_f(ref, x, F, ref=True)
            manifest.append({"key": key, "F": F})
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "viterbi_golden.npz"), **arrays)
    print("wrote", len(manifest), "cases")


if __name__ == "__main__":
    main()
