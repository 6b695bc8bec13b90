"""C3 coded traffic (1024 subframes, 20 dB) on two lanes (HIP streams), driven serially from one host
thread or with one host thread per lane, for repeated (rotate 1) and changing (rotate 4) descriptors:
ms per 1024-subframe batch and host seconds per step."""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "empower-srslte_amd"))


def main():
    import torch
    import srsgpu_traffic as tr
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    out = {}
    steps = 40
    for rotate in (1, 4):
        ms = [tr.MixedCells(table, 1024, torch, dev, seed=22, stream=streams[li].cuda_stream, snr_db=20.0, prbs=(100,),
                            mcs=28, full_band=True, keep=list(range(li, 1024, 2)), rotate=rotate) for li in range(2)]
        for mode in ("serial", "threaded", "serial", "threaded"):
            for _ in range(10):
                for m in ms:
                    m.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "serial":
                for _ in range(steps):
                    for m in ms:
                        m.step()
            else:
                def run(m):
                    for _ in range(steps):
                        m.step()
                th = [threading.Thread(target=run, args=(m,)) for m in ms]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            out.setdefault("rotate%d_%s" % (rotate, mode), []).append(round(el / steps * 1e3, 3))
        acks = [m.check()[0] for m in ms]
        out["rotate%d_acks" % rotate] = acks
        for m in ms:
            m.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
