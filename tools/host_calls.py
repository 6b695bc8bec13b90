"""Host (enqueue) time of each call of the C3 receive step, one lane of 512 subframes: OFDM, chest,
PDSCH LLRs, softbuffer reset, DL-SCH decode. rotate 1 repeats the same descriptors (the engines'
repeat-call caches hit); rotate 4 cycles four descriptor sets (a receiver whose grants change).
sync: synchronise after every step (the calls' own host cost, no queue back-pressure)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))


def main():
    import torch
    import srsgpu_phy as s
    import srsgpu_traffic as tr
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    dev = torch.device("cuda", 0)
    out = {}
    for rotate in (1, 4):
        st = torch.cuda.Stream(dev)
        m = tr.MixedCells(table, 512, torch, dev, seed=22, stream=st.cuda_stream, snr_db=20.0, prbs=(100,), mcs=28,
                          full_band=True, rotate=rotate)
        c = m.cells[0]
        n, gsz, N = c["n"], c["gsz"], c["N"]
        calls = {
            "ofdm": lambda: c["ofdm"].rx_dev(n, c["x"].data_ptr(), 15 * N, c["grid"].data_ptr(), gsz),
            "chest": lambda: c["chest"].estimate_dev(c["sf_idx"], c["grid"].data_ptr(), gsz, c["ce"].data_ptr(),
                                                     c["noise"].data_ptr()),
            "llr": lambda: c["pd"].llr_dev(c["sfs_rot"][m.cur], c["grid"].data_ptr(), c["ce"].data_ptr(), gsz,
                                           m.d_e.data_ptr(), c["e_offs"]),
            "reset": lambda: m.dlsch.reset_range(m.cur * m.ntb, m.ntb),
            "decode": lambda: m.dlsch.decode_dev(m.tb_rot[m.cur], m.d_e.data_ptr(), m.d_data.data_ptr(), 8,
                                                 m.d_ret.data_ptr(), m.d_noi.data_ptr()),
        }
        for sync in (True, False):
            acc = {k: [] for k in calls}
            for it in range(40):
                m.cur = (m.cur + 1) % rotate
                for k, f in calls.items():
                    t0 = time.perf_counter()
                    r = f()
                    acc[k].append(time.perf_counter() - t0)
                    assert r in (0, None), (k, r)
                if sync:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
            out["rotate%d_%s" % (rotate, "sync" if sync else "async")] = {
                k: round(float(np.median(v[5:])) * 1e3, 4) for k, v in acc.items()}
        m.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
