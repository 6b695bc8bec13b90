"""Record golden extended-CP vectors (SRSLTE_CP_EXT: 6 OFDM symbols per slot) from the reference
build (`make -C oracle ref`):
  - PDSCH RE orders, srslte_pdsch_get (pdsch.c:95-234) over an index-valued 12-symbol grid;
  - PDCCH REG orders and NOF_CCE, srslte_regs_init / srslte_regs_pdcch_get (regs.c:587-616: symbol 3
    of a 4-symbol control region carries CRS);
  - CRS pilots, srslte_refsignal_cs_set_cell (refsignal_dl.c:265-318 with N_cp = 0, l' = 3);
  - channel estimates, noise and measurements of chest_dl.c itself (oracle/_ref/ref_front) on random
    12-symbol grids: per-symbol (time interpolation chest_dl.c:433-441) and averaged estimation, REFS /
    PSS / EMPTY noise, ports 0-3.

    python tests/golden/make_extcp_golden.py   -> tests/golden/extcp_golden.npz
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import Ref, pdcch_map, ref_front_chest  # noqa: E402

EXT = 256  # nof_ports flag of the oracle / harness entry points: extended CP


def main():
    ref = Ref()
    rng = np.random.default_rng(612)
    arrays, man = {}, dict(re_maps=[], pdcch_maps=[], crs=[], chest=[])
    get = ref.lib.ref_pdsch_get
    get.argtypes = [ctypes.c_uint32] * 5 + [ctypes.c_void_p] * 3
    for nof_prb in (6, 15, 25, 50, 75, 100):
        for nports in (1, 2, 4):
            cell_id = int(rng.integers(0, 504))
            for sf_idx, lstart in ((0, 1), (5, 2), (1, 3), (0, 4)):
                mask = (rng.random((2, nof_prb)) < 0.7).astype(np.uint8)
                g = np.arange(12 * 12 * nof_prb).astype(np.complex64)
                out = np.zeros(12 * 12 * nof_prb, np.complex64)
                n = get(nof_prb, cell_id, nports | EXT, lstart, sf_idx, mask.ctypes.data, g.ctypes.data, out.ctypes.data)
                key = "re%d" % len(man["re_maps"])
                arrays[key] = out[:n].real.astype(np.uint32)
                arrays[key + "_mask"] = mask
                man["re_maps"].append(dict(key=key, nof_prb=nof_prb, cell_id=cell_id, nports=nports, sf_idx=sf_idx,
                                           lstart=lstart))
    for nof_prb in (6, 7, 10, 15, 25, 100):
        for nports in (1, 2, 4):
            cell_id = int(rng.integers(0, 504))
            pl, pr = int(rng.integers(0, 2)), int(rng.integers(0, 4))
            for cfi in (1, 2, 3):
                idx, ncce = pdcch_map(ref, nof_prb, cell_id, nports | EXT, pl, pr, cfi, ref=True)
                key = "pm%d" % len(man["pdcch_maps"])
                arrays[key] = idx
                man["pdcch_maps"].append(dict(key=key, nof_prb=nof_prb, cell_id=cell_id, nports=nports, phich_len=pl,
                                              phich_res=pr, cfi=cfi, nof_cce=ncce))
    pil = ref.lib.ref_crs_pilots_cp
    pil.argtypes = [ctypes.c_uint32] * 5 + [ctypes.c_void_p]
    for nof_prb, cell_id in ((6, 0), (25, 151), (100, 503)):
        for sf_idx in range(10):
            for pair in (0, 1):
                o = np.zeros((4 if pair == 0 else 2) * 2 * nof_prb, np.complex64)
                assert pil(nof_prb, cell_id, 1, pair, sf_idx, o.ctypes.data) == 0
                key = "crs%d" % len(man["crs"])
                arrays[key] = o
                man["crs"].append(dict(key=key, nof_prb=nof_prb, cell_id=cell_id, sf_idx=sf_idx, pair=pair))
    sym = {6: 128, 15: 256, 25: 384, 50: 768, 100: 1536}
    cases = [(6, 1, 1, dict()), (6, 4, 2, dict(average=True)), (15, 2, 2, dict(noise_alg=1)),
             (25, 1, 2, dict(average=True, noise_alg=2)), (25, 4, 1, dict(gauss=(4, 1.0), smooth_auto=True)),
             (50, 2, 1, dict(average=True, gauss=(4, 1.0))), (100, 1, 1, dict(noise_alg=1, average=True))]
    for nof_prb, nports, nrx, cfg in cases:
        cell_id = int(rng.integers(0, 504))
        sfs = [0, 1, 5] if nof_prb < 50 else [5]
        n = 12 * 12 * nof_prb
        grids = [[(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for _ in range(nrx)]
                 for _ in sfs]
        out = ref_front_chest(nof_prb, cell_id, nports, nrx, sfs, grids, cp=1, noise_init=0.05, **cfg)
        key = "ch%d" % len(man["chest"])
        for i in range(len(sfs)):
            for a in range(nrx):
                arrays["%s_%d_y%d" % (key, i, a)] = grids[i][a]
            r = out[i]
            arrays["%s_%d_ce" % (key, i)] = r["ce"]
            for f in ("noise", "rsrp", "rssi", "rsrp_corr", "cfo"):
                arrays["%s_%d_%s" % (key, i, f)] = r[f]
        man["chest"].append(dict(key=key, nof_prb=nof_prb, cell_id=cell_id, nports=nports, nrx=nrx, sfs=sfs,
                                 symbol_sz=sym[nof_prb], average=bool(cfg.get("average", False)),
                                 noise_alg=cfg.get("noise_alg", 0), gauss=cfg.get("gauss"),
                                 smooth_auto=bool(cfg.get("smooth_auto", False)), noise_init=0.05))
    arrays["manifest"] = np.frombuffer(json.dumps(man).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "extcp_golden.npz"), **arrays)
    print({k: len(v) for k, v in man.items()})


if __name__ == "__main__":
    main()
