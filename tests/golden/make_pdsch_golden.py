"""Record golden PDSCH front-end vectors from the srsLTE reference (oracle/_ref: pdsch.c,
precoding.c, demod_soft.c, sequence.c, scrambling.c compiled from the reference's sources):
RE-extraction index lists (srslte_pdsch_get on an index-valued grid), SISO equaliser outputs
(srslte_predecoding_single_multi, with and without CSI), int16 soft demapper outputs for all
modulations and the PDSCH-scrambled LLRs.

    python tests/golden/make_pdsch_golden.py   -> tests/golden/pdsch_golden.npz
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import Ref, ref_pdsch  # noqa: E402

f32 = ctypes.POINTER(ctypes.c_float)
i16 = ctypes.POINTER(ctypes.c_int16)
u8 = ctypes.POINTER(ctypes.c_uint8)


def main():
    L = ref_pdsch(Ref())
    rng = np.random.default_rng(36211)
    arrays, man = {}, []
    # RE maps: (nof_prb, cell_id, ports, lstart, sf_idx, mask kind)
    for k, (nprb, cid, ports, lstart, sf, kind) in enumerate([
            (100, 1, 1, 1, 1, "all"), (100, 1, 1, 1, 0, "all"), (100, 301, 2, 2, 5, "all"),
            (25, 17, 1, 3, 0, "all"), (25, 5, 4, 2, 5, "random"), (6, 0, 1, 4, 0, "all"),
            (15, 100, 2, 3, 0, "slots"), (50, 77, 1, 2, 9, "random"), (75, 11, 1, 1, 0, "all")]):
        if kind == "all":
            mask = np.ones((2, nprb), np.uint8)
        elif kind == "random":
            mask = (rng.random((2, nprb)) < 0.5).astype(np.uint8)
        else:
            m = (rng.random(nprb) < 0.5).astype(np.uint8)
            mask = np.stack([m, m])
        grid = np.zeros(nprb * 12 * 14, np.complex64)
        grid.real = np.arange(grid.size)
        out = np.zeros(grid.size, np.complex64)
        n = L.ref_pdsch_get(nprb, cid, ports, lstart, sf, mask.ctypes.data_as(u8),
                            grid.ctypes.data_as(f32), out.ctypes.data_as(f32))
        key = "map%02d" % k
        arrays[key + "_mask"] = mask
        arrays[key + "_idx"] = out[:n].real.astype(np.uint32)
        man.append(dict(key=key, kind="map", nof_prb=nprb, cell_id=cid, ports=ports, lstart=lstart,
                        sf_idx=sf))
    # equaliser
    for k, (n, noise, csi) in enumerate([(4099, 0.0, 0), (4099, 0.05, 0), (1037, 0.1, 0),
                                         (1037, 0.1, 1), (33, 0.0, 1)]):
        y = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        h = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        x = np.zeros_like(y)
        c = np.zeros(n, np.float32)
        L.ref_predecode_single(y.ctypes.data_as(f32), h.ctypes.data_as(f32), x.ctypes.data_as(f32),
                               c.ctypes.data_as(f32) if csi else None, n, 1.0, noise)
        key = "eq%02d" % k
        arrays[key + "_y"], arrays[key + "_h"], arrays[key + "_x"] = y, h, x
        if csi:
            arrays[key + "_csi"] = c
        man.append(dict(key=key, kind="eq", n=n, noise=noise, csi=csi))
    # soft demapper (incl. SIMD tails and saturating inputs)
    for k, (mod, n, sc) in enumerate([(1, 4001, 1.0), (1, 1003, 200.0), (2, 4001, 1.0),
                                      (2, 1003, 100.0), (3, 4001, 1.0), (3, 1003, 60.0),
                                      (0, 100, 1.0)]):
        s = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * sc).astype(np.complex64)
        bps = {0: 1, 1: 2, 2: 4, 3: 6}[mod]
        llr = np.zeros(n * bps, np.int16)
        L.ref_demod_s(mod, s.ctypes.data_as(f32), n, llr.ctypes.data_as(i16))
        key = "dm%02d" % k
        arrays[key + "_sym"], arrays[key + "_llr"] = s, llr
        man.append(dict(key=key, kind="demod", mod=mod, n=n))
    # scrambling
    for k, (rnti, q, nslot, cid, n) in enumerate([(1234, 0, 2, 1, 30000), (65535, 1, 18, 503, 5000)]):
        x = rng.integers(-32768, 32768, n).astype(np.int16)
        y = x.copy()
        L.ref_scramble_pdsch_s(rnti, q, nslot, cid, y.ctypes.data_as(i16), n)
        key = "sc%02d" % k
        arrays[key + "_in"], arrays[key + "_out"] = x, y
        man.append(dict(key=key, kind="scramble", rnti=rnti, q=q, nslot=nslot, cell_id=cid, n=n))
    arrays["manifest"] = np.frombuffer(json.dumps(man).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "pdsch_golden.npz"), **arrays)
    print(len(man), "cases")


if __name__ == "__main__":
    main()
