"""Record golden TM2 transmit-diversity vectors (2 ports: srslte_predecoding_type with
SRSLTE_MIMO_TYPE_TX_DIVERSITY, precoding.c:1811-1818 -> srslte_predecoding_diversity_multi, then
srslte_layerdemap_type, layermap.c:175-) from the reference build (`make -C oracle ref`): RE counts
below and above the 32-RE SSE threshold and not multiples of 4 (SSE body + C tail), 1 and 2 rx
antennas, CSI on and off, scaling 1 and rho_a-like, a pair with an all-zero channel; and the
4-port form (RE quadruplets, ports 0/2 and 1/3) at RE counts 4 .. 1200.

    python tests/golden/make_txdiv_golden.py   -> tests/golden/txdiv_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import Ref, predecode_txdiv  # noqa: E402


def main():
    ref = Ref()
    rng = np.random.default_rng(2026)
    arrays, manifest = {}, []
    for n in (6, 32, 34, 38, 120, 1202):
        for nrx in (1, 2):
            for csi in (False, True):
                sc = 1.0 if n % 4 else 0.7079
                key = "tx_%d_%d_%d" % (n, nrx, int(csi))
                y = [(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
                h = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
                     for _ in range(2)]
                h[0][0][2:4] = 0
                h[1][0][2:4] = 0
                out = predecode_txdiv(ref, y, h, sc, csi, ref=True)
                d, c = out if csi else (out, None)
                for a in range(nrx):
                    arrays[key + "_y%d" % a] = y[a]
                    for p in range(2):
                        arrays[key + "_h%d%d" % (p, a)] = h[p][a]
                arrays[key + "_d"] = d
                if csi:
                    arrays[key + "_csi"] = c
                manifest.append({"key": key, "n": n, "nrx": nrx, "csi": csi, "scaling": sc})
    # 4 ports (precoding.c:388-423, 604-662): RE quadruplets, no SSE form, no zero guard (so no
    # all-zero channel here: the reference divides by 0)
    for n in (4, 36, 120, 1200):
        for nrx in (1, 2):
            for csi in (False, True):
                sc = 1.0 if n % 8 else 0.7079
                key = "tx4_%d_%d_%d" % (n, nrx, int(csi))
                y = [(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
                h = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
                     for _ in range(4)]
                out = predecode_txdiv(ref, y, h, sc, csi, ref=True)
                d, c = out if csi else (out, None)
                for a in range(nrx):
                    arrays[key + "_y%d" % a] = y[a]
                    for p in range(4):
                        arrays[key + "_h%d%d" % (p, a)] = h[p][a]
                arrays[key + "_d"] = d
                if csi:
                    arrays[key + "_csi"] = c
                manifest.append({"key": key, "n": n, "nrx": nrx, "csi": csi, "scaling": sc, "ports": 4})
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "txdiv_golden.npz"), **arrays)
    print("wrote", len(manifest), "cases")


if __name__ == "__main__":
    main()
