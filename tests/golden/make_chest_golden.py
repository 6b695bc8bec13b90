"""Record golden channel estimates from the reference's own chest_dl.c (oracle/_ref/ref_front, built by
`make -C oracle ref` in the build container; chest_dl.c / pss.c / convolution.c / interp.c compiled where
they lie, srslte_dft_* left unresolved because the estimation path never calls them).

Each case runs ONE reference estimator (srslte_chest_dl_init / set_cell and srsUE's setters,
srsue/src/phy/phch_worker.cc:148-150, 553-565) over a sequence of subframes, so the PSS / EMPTY noise
state carries between subframes as in srsUE. Recorded per subframe: the input grids, the noise estimate
the object held before the call, the CE grids of every (rx antenna, port), noise / RSRP / RSSI / RSRP
correlation / CFO per (rx antenna, port) and the getters (srslte_chest_dl_get_*).

    python tests/golden/make_chest_golden.py   -> tests/golden/chest_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from chest_synth import sync_grid  # noqa: E402
from srsgpu_testlib import ref_front_chest  # noqa: E402

# (name, nof_prb, cell_id, nports, nrx, sfs, filt, gauss, smooth_auto, average, noise_alg, noise_init)
CASES = [
    # srsUE's defaults (main.cc:287-301): average_subframe, Gaussian order 4 / std 1, REFS noise,
    # neighbour RSRP, CFO on every subframe
    ("srsue_6_2x2", 6, 3, 2, 2, list(range(10)), (), (4, 1.0), False, True, 0, 0.0),
    ("srsue_25_1x1", 25, 1, 1, 1, list(range(10)), (), (4, 1.0), False, True, 0, 0.0),
    ("srsue_100_1x2", 100, 7, 1, 2, [0, 1], (), (4, 1.0), False, True, 0, 0.0),
    ("srsue_50_2x1", 50, 500, 2, 1, [4, 5], (), (4, 1.0), False, True, 0, 0.0),
    # time interpolation between the CRS symbols with the default 3-tap filter
    ("interp_25_2x1", 25, 11, 2, 1, [0, 1, 5], (0.1, 0.8, 0.1), None, False, False, 0, 0.0),
    ("interp_15_1x2", 15, 503, 1, 2, [9, 0], (0.1, 0.8, 0.1), None, False, False, 0, 0.0),
    # PSS / EMPTY noise: estimated in subframes 0 and 5 only, carried otherwise
    ("pss_25_2x2", 25, 4, 2, 2, [3, 4, 5, 6], (), (4, 1.0), False, True, 1, 0.004),
    ("empty_15_1x2", 15, 2, 1, 2, [4, 5, 6], (0.05, 0.2, 0.5, 0.2, 0.05), None, False, False, 2, 0.004),
    ("pss_interp_6_1x1", 6, 9, 1, 1, [0, 1, 2], (0.1, 0.4, 0.4, 0.1), None, False, False, 1, 0.01),
    # smooth_filter_auto (Gaussian from the noise estimate, chest_dl.c:616-618)
    ("auto_25_1x1", 25, 8, 1, 1, [0, 1, 2], (), (4, 1.0), True, False, 0, 0.0),
    ("auto_avg_25_2x1", 25, 8, 2, 1, [2, 3], (), (4, 1.0), True, True, 0, 0.0),
    # no smoothing: the average_subframe quirk (raw pilot buffer interpolated, chest_dl.c:619-621)
    ("nosmooth_avg_25_1x1", 25, 301, 1, 1, [1, 5], (), None, False, True, 0, 0.0),
    ("nosmooth_6_1x1", 6, 0, 1, 1, [7], (), None, False, False, 0, 0.0),
    # 4 CRS ports: ports 2 / 3 in symbols 1 and 8 (refsignal_dl.c:76-122), their 2-symbol time
    # interpolation (chest_dl.c:427-431), noise and averaging over 2 symbols, and the CFO reading
    # port 1's rows of the shared pilot buffer
    ("srsue_25_4x2", 25, 5, 4, 2, [0, 1, 5], (), (4, 1.0), False, True, 0, 0.0),
    ("interp_50_4x1", 50, 13, 4, 1, [2, 5], (0.1, 0.8, 0.1), None, False, False, 0, 0.0),
    ("pss_6_4x2", 6, 8, 4, 2, [4, 5, 6], (), (4, 1.0), False, True, 1, 0.004),
    ("nosmooth_avg_15_4x1", 15, 2, 4, 1, [3], (), None, False, True, 0, 0.0),
    ("auto_25_4x1", 25, 20, 4, 1, [1], (), (4, 1.0), True, False, 0, 0.0),
    ("empty_interp_6_4x1", 6, 1, 4, 1, [0, 7], (0.05, 0.2, 0.5, 0.2, 0.05), None, False, False, 2, 0.004),
]


def main():
    rng = np.random.default_rng(2024)
    arrays, man = {}, []
    for name, nof_prb, cell_id, nports, nrx, sfs, filt, gauss, auto, average, alg, noise_init in CASES:
        grids = [[sync_grid(nof_prb, cell_id, sf, nports, rng, flat=average) for _ in range(nrx)] for sf in sfs]
        res = ref_front_chest(nof_prb, cell_id, nports, nrx, sfs, grids, filt=filt, gauss=gauss, smooth_auto=auto,
                              average=average, noise_alg=alg, noise_init=noise_init)
        arrays[name + "_grid"] = np.array(grids, np.complex64)                          # [sf][rx][n]
        arrays[name + "_ce"] = np.array([r["ce"] for r in res], np.complex64)          # [sf][rx][port][n]
        for k in ("noise_before", "noise", "rsrp", "rssi", "rsrp_corr", "cfo"):
            arrays[name + "_" + k] = np.array([r[k] for r in res], np.float32)         # [sf][rx][port]
        arrays[name + "_getters"] = np.array([r["getters"] for r in res], np.float32)
        man.append(dict(name=name, nof_prb=nof_prb, cell_id=cell_id, nports=nports, nrx=nrx, sfs=sfs,
                        filt=list(filt), gauss=list(gauss) if gauss else None, smooth_auto=auto, average=average,
                        noise_alg=alg, noise_init=noise_init))
    arrays["manifest"] = np.frombuffer(json.dumps(man).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "chest_golden.npz"), **arrays)
    print("%d cases, %d subframes" % (len(man), sum(len(c["sfs"]) for c in man)))


if __name__ == "__main__":
    main()
