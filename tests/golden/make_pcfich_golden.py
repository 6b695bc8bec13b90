"""Record golden PCFICH decodes from the reference build (`make -C oracle ref`): the reference's
srslte_regs_init + srslte_pcfich_init/set_cell + srslte_pcfich_decode_multi (pcfich.c:178-241) on
synthetic symbol-0 grids: CFI codewords scrambled, QPSK-modulated, sent through random flat-ish
channels (1, 2 or 4 ports; 2 ports as SFBC pairs, 4 as SFBC quadruplets) at SNRs from hopeless to
clean, with and without
the noise estimate. Only OFDM symbol 0 is stored (the rest of the subframe is zero and unread).

    python tests/golden/make_pcfich_golden.py   -> tests/golden/pcfich_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import Ref, pcfich_decode, pcfich_re_map  # noqa: E402

CW = [[0, 1, 1], [1, 0, 1], [1, 1, 0]]  # 36.212 Table 5.3.4-1, repeated to 32 bits


def gold(c_init, n):
    x1 = np.zeros(1600 + n + 31, np.uint8)
    x2 = np.zeros_like(x1)
    x1[0] = 1
    x2[:31] = [(c_init >> i) & 1 for i in range(31)]
    for k in range(1600 + n):
        x1[k + 31] = x1[k + 3] ^ x1[k]
        x2[k + 31] = x2[k + 3] ^ x2[k + 2] ^ x2[k + 1] ^ x2[k]
    return (x1[1600:1600 + n] ^ x2[1600:1600 + n]).astype(np.uint8)


def synth(rng, nof_prb, cell_id, nports, nrx, sf_idx, cfi, snr_db, idx):
    """symbol-0 grids y[a] and estimates h[p][a] (nof_prb*12 complex64 each)"""
    n0 = nof_prb * 12
    b = np.array([CW[cfi - 1][i % 3] for i in range(32)], np.uint8)
    b ^= gold((sf_idx + 1) * (2 * cell_id + 1) * 512 + cell_id, 32)
    x = ((1 - 2.0 * b[0::2]) + 1j * (1 - 2.0 * b[1::2])) / np.sqrt(2)
    sig = 10 ** (-snr_db / 20)
    h = [[(rng.standard_normal(n0) + 1j * rng.standard_normal(n0)).astype(np.complex64) * 0.7
          for _ in range(nrx)] for _ in range(nports)]
    y = []
    for a in range(nrx):
        g = np.zeros(n0, np.complex128)
        if nports == 1:
            g[idx] = h[0][a][idx] * x
        elif nports == 4:  # quadruplets (precoding.c:1863-1889): ports 0/2 on k0, k1, ports 1/3 on k2, k3
            for i in range(4):
                k = idx[4 * i:4 * i + 4]
                x0, x1, x2, x3 = x[4 * i:4 * i + 4]
                g[k[0]] = (h[0][a][k[0]] * x0 - h[2][a][k[0]] * np.conj(x1)) / np.sqrt(2)
                g[k[1]] = (h[0][a][k[1]] * x1 + h[2][a][k[1]] * np.conj(x0)) / np.sqrt(2)
                g[k[2]] = (h[1][a][k[2]] * x2 - h[3][a][k[2]] * np.conj(x3)) / np.sqrt(2)
                g[k[3]] = (h[1][a][k[3]] * x3 + h[3][a][k[3]] * np.conj(x2)) / np.sqrt(2)
        else:  # SFBC: pair (k0, k1) carries (x0, x1) on port 0 and (-x1*, x0*) on port 1
            for i in range(8):
                k0, k1 = idx[2 * i], idx[2 * i + 1]
                x0, x1 = x[2 * i], x[2 * i + 1]
                g[k0] = (h[0][a][k0] * x0 - h[1][a][k0] * np.conj(x1)) / np.sqrt(2)
                g[k1] = (h[0][a][k1] * x1 + h[1][a][k1] * np.conj(x0)) / np.sqrt(2)
        g += sig * (rng.standard_normal(n0) + 1j * rng.standard_normal(n0)) / np.sqrt(2)
        y.append(g.astype(np.complex64))
    return y, h


def main():
    ref = Ref()
    rng = np.random.default_rng(2024)
    arrays, manifest = {}, []
    k = 0
    for nof_prb in (6, 15, 25, 50, 75, 100):
        for nports in (1, 2):
            for nrx in (1, 2):
                for rep in range(3):
                    cell_id = int(rng.integers(0, 504))
                    sf_idx = int(rng.integers(0, 10))
                    cfi = int(rng.integers(1, 4))
                    snr = float(rng.choice([-10.0, 0.0, 5.0, 20.0]))
                    noise = float(rng.choice([0.0, 10 ** (-snr / 10)]))
                    idx = pcfich_re_map(ref, nof_prb, cell_id, ref=True)
                    y, h = synth(rng, nof_prb, cell_id, nports, nrx, sf_idx, cfi, snr, idx)
                    got = pcfich_decode(ref, nof_prb, cell_id, nports, nrx, y, h, noise, sf_idx, ref=True)
                    key = "p%d" % k
                    k += 1
                    for a in range(nrx):
                        arrays["%s_y%d" % (key, a)] = y[a]
                        for p in range(nports):
                            arrays["%s_h%d%d" % (key, p, a)] = h[p][a]
                    arrays[key + "_idx"] = idx
                    manifest.append({"key": key, "nof_prb": nof_prb, "cell_id": cell_id, "nports": nports,
                                     "nrx": nrx, "sf_idx": sf_idx, "noise": noise, "sent_cfi": cfi,
                                     "snr_db": snr, "cfi": got[0], "corr": got[1]})
    rng4 = np.random.default_rng(4444)  # 4 CRS ports, after the cases above
    for nof_prb in (6, 15, 25, 50, 75, 100):
        for nrx in (1, 2):
            for rep in range(2):
                cell_id = int(rng4.integers(0, 504))
                sf_idx = int(rng4.integers(0, 10))
                cfi = int(rng4.integers(1, 4))
                snr = float(rng4.choice([-10.0, 0.0, 5.0, 20.0]))
                noise = float(rng4.choice([0.0, 10 ** (-snr / 10)]))
                idx = pcfich_re_map(ref, nof_prb, cell_id, ref=True)
                y, h = synth(rng4, nof_prb, cell_id, 4, nrx, sf_idx, cfi, snr, idx)
                got = pcfich_decode(ref, nof_prb, cell_id, 4, nrx, y, h, noise, sf_idx, ref=True)
                key = "p%d" % k
                k += 1
                for a in range(nrx):
                    arrays["%s_y%d" % (key, a)] = y[a]
                    for p in range(4):
                        arrays["%s_h%d%d" % (key, p, a)] = h[p][a]
                arrays[key + "_idx"] = idx
                manifest.append({"key": key, "nof_prb": nof_prb, "cell_id": cell_id, "nports": 4,
                                 "nrx": nrx, "sf_idx": sf_idx, "noise": noise, "sent_cfi": cfi,
                                 "snr_db": snr, "cfi": got[0], "corr": got[1]})
    arrays["manifest"] = np.frombuffer(json.dumps(manifest).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "pcfich_golden.npz"), **arrays)
    ok = sum(m["cfi"] == m["sent_cfi"] for m in manifest)
    print("wrote", len(manifest), "cases;", ok, "decode the sent CFI")


if __name__ == "__main__":
    main()
