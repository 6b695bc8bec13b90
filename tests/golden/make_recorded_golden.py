"""Fixtures from the reference's own over-the-air recordings (lib/src/phy/phch/test/, the inputs of its
ctest cases, CMakeLists.txt:213-216):

  signal.10M.dat         pcfich_file_test -c 150 -n 50 -p 2: cell 150, 50 PRB (N = 1024), 2 CRS ports;
                         the file holds 7681 samples, half a subframe: srslte_ofdm_init_ zeroes the
                         input buffer (ofdm.c:84-88), so the rest of the subframe is zeros. Pass
                         criterion (pcfich_file_test.c:244-256): CFI 1 with correlation > 2.8.
  signal.1.92M.amar.dat  pdsch_pdcch_file_test / pdcch_file_test -c 1 -n 6 -p 1: cell 1, 6 PRB (N = 128),
                         1 port, 10 subframes from sf_idx 0, SI-RNTI. Pass criterion
                         (pdsch_pdcch_file_test.c:186-210): srslte_ue_dl_decode returns > 0 (a DCI found and
                         its PDSCH decoded) in one of the subframes.

The recordings themselves are stored as fixture data (complex64 samples). The expected outputs come from
the reference: the received grids of the numpy OFDM oracle (oracle/ofdm_oracle.py: FFTW is absent, so
the reference's srslte_ofdm_rx_sf cannot run here) go through oracle/_ref/ref_front ue_dl, i.e. the
reference's chest_dl.c, pcfich.c, pdcch.c, ue_dl.c's DCI search, dci.c / ra.c and pdsch.c, in
srslte_ue_dl_decode_rnti's order. Recorded per subframe: CFI, correlation, noise estimate, the DL search
result (format, location, message bits), return value, TBS, rv, modulation, ack, nof_iterations,
RE count, TB bytes, and the channel estimates.

    python tests/golden/make_recorded_golden.py   -> tests/golden/recorded_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import ofdm_oracle as oo  # noqa: E402
from srsgpu_testlib import ref_front_ue_dl  # noqa: E402

SRC = "/root/reference/lib/src/phy/phch/test"
SIRNTI = 0xFFFF
# name: (file, nof_prb, cell_id, nports, N, subframes, phich (length, resources), max_prb)
CASES = {
    "s10m": ("signal.10M.dat", 50, 150, 2, 1024, 1, (0, 2), 50),
    "amar": ("signal.1.92M.amar.dat", 6, 1, 1, 128, 10, (0, 2), 6),
}


def grids_of(x, nof_prb, N, nsf):
    """the time samples split into subframes of 15 N (zero-padded as the reference's zeroed input
    buffer leaves a short read) -> numpy OFDM grids [nsf][14 * 12 nof_prb]"""
    L = 15 * N
    pad = np.zeros(nsf * L, np.complex64)
    pad[:min(x.size, pad.size)] = x[:pad.size]
    return [oo.rx_sf(pad[i * L:(i + 1) * L], nof_prb, N).reshape(-1).astype(np.complex64) for i in range(nsf)]


def main():
    arrays, man = {}, {}
    for name, (fname, nof_prb, cell_id, nports, N, nsf, (pl, pr), max_prb) in CASES.items():
        x = np.fromfile(os.path.join(SRC, fname), np.complex64)
        g = grids_of(x, nof_prb, N, nsf)
        res = ref_front_ue_dl(nof_prb, cell_id, nports, 1, pl, pr, max_prb, SIRNTI, 0, list(range(nsf)),
                              [[gi] for gi in g])
        arrays[name + "_x"] = x
        for k in ("cfi", "corr", "noise", "ret", "tbs", "rv", "mod", "ack", "noi", "nre"):
            arrays["%s_%s" % (name, k)] = np.array([r[k] for r in res])
        arrays[name + "_dl"] = np.array([r["dl"][:5] for r in res], np.int32)
        arrays[name + "_msg"] = np.stack([np.pad(r["dl"][5], (0, 128 - r["dl"][5].size)) for r in res])
        arrays[name + "_data"] = np.stack([r["data"][:max(1, max(rr["tbs"] for rr in res) // 8)] for r in res])
        arrays[name + "_ce"] = np.stack([r["ce"] for r in res])
        man[name] = dict(file=fname, nof_prb=nof_prb, cell_id=cell_id, nof_ports=nports, N=N, subframes=nsf,
                         phich_length=pl, phich_resources=pr, max_prb=max_prb, rnti=SIRNTI, tm=0,
                         samples=int(x.size))
        print(name, [(r["cfi"], round(r["corr"], 3), r["dl"][0], r["ret"], r["ack"]) for r in res])
    arrays["manifest"] = np.frombuffer(json.dumps(man).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "recorded_golden.npz"), **arrays)


if __name__ == "__main__":
    main()
