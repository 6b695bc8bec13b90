"""Lifecycle of the queue's zero-copy host memory (VERDICT r5 "next" 1; the bench's r05_s39 / r05_s46
fault came at the first pageable hipMemcpy after a closed queue's registered output block had been
unregistered and freed).

Each cycle creates a queue, puts the samples and the TB outputs in zero-copy host memory, decodes a
batch of coded 20 MHz subframes through it (native worker threads, TB bytes written into that memory
by the decoder), closes the queue, frees the memory, then allocates memory of the same size again
(usually at the same addresses), copies it to the device with plain pageable copies (torch H2D and a
DL-SCH engine's CRC-table upload, the call that faulted) and checks the bytes — and the next cycle's
queue decodes again. Queue-owned blocks (srsgpu_rxq_alloc_host, the bench's form) and caller memory
(srsgpu_rxq_register / unregister, then munmap) both; and the queue refuses to unpin or free the
other kind."""
import json
import mmap
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C3_TBS = 75376


@pytest.fixture(scope="module")
def c3():
    import torch
    import srsgpu_traffic as tr
    dev = torch.device("cuda:0")
    table = json.load(open(os.path.join(REPO, "tests", "golden", "c5_traffic.json")))
    m = tr.MixedCells(table, 32, torch, dev, seed=22, snr_db=30.0, prbs=(100,), mcs=28, full_band=True)
    c = m.cells[0]
    x = c["x"].cpu().numpy().reshape(c["n"], 15 * c["N"])
    tx = m.d_data_tx.cpu().numpy()
    want = [tx[t["data_offset"]:t["data_offset"] + C3_TBS // 8] for t in m.tb_list]
    out = {"N": c["N"], "n": c["n"], "x": x, "sfs": c["sfs"], "want": want}
    m.close()
    torch.cuda.synchronize()
    scale = float(np.abs(x.view(np.float32)).max()) / 32000.0
    out["sc"] = np.round(x.view(np.float32) / scale).astype(np.int16)
    out["scale"] = scale
    return out


def _cycle(s, torch, c3, mode, nsb=48):
    q = s.RxQueue(100, 1, c3["N"], nof_softbuffers=nsb, max_batch=16, max_wait_us=800)
    q.set_input_format(q.SC16, c3["scale"])
    dl = (C3_TBS // 8 + 6 + 63) // 64 * 64
    mm = None
    if mode == "owned":
        src = q.alloc_host(c3["sc"].shape, np.int16)
        src[...] = c3["sc"]
        block = q.alloc_host((nsb, dl), np.uint8)
    else:
        src = c3["sc"].copy()
        q.register(src)
        mm = mmap.mmap(-1, nsb * dl)
        block = np.frombuffer(mm, np.uint8).reshape(nsb, dl)
        q.register(block)
    addr, nbytes = block.ctypes.data, block.nbytes
    outs = [block[k, :C3_TBS // 8 + 6] for k in range(nsb)]
    items = []
    for i in range(nsb):
        j = i % c3["n"]
        sf = c3["sfs"][j]
        sf.softbuffer[0] = i
        items.append(q.item([src[j]], sf, [outs[i]]))
    _, _, status = q.drive(items, 4)
    assert (status == 0).all()
    for i in range(nsb):
        assert items[i].ret[0] == 0, i
        assert (outs[i][:C3_TBS // 8] == c3["want"][i % c3["n"]]).all(), i
    if mode == "owned":
        with pytest.raises(RuntimeError):  # a queue-owned block is not the caller's to unpin
            q.unregister(block)
    else:
        with pytest.raises(RuntimeError):  # nor caller memory the queue's to free
            q.free_host(block)
        q.unregister(block)
        q.unregister(src)
    del items, outs, block, src
    q.close()
    torch.cuda.synchronize()
    if mm is not None:
        mm.close()  # munmap of the pages the queue had pinned
    # the same size again (usually the same addresses), plain pageable copies from it
    mm2 = mmap.mmap(-1, nbytes)
    a = np.frombuffer(mm2, np.uint8)
    a[:] = (np.arange(a.size) * 7).astype(np.uint8)
    d = torch.from_numpy(a).to("cuda")
    assert (d.cpu().numpy() == a).all()
    dlsch = s.Dlsch(8)  # its CRC-table upload is a pageable hipMemcpy of 1.6 MB
    dlsch.close()
    torch.cuda.synchronize()
    same = a.ctypes.data == addr
    del a, d
    mm2.close()
    return same


@pytest.mark.parametrize("mode", ["owned", "registered"])
def test_zero_copy_memory_lifecycle(c3, mode):
    import torch
    import srsgpu_phy as s
    for _ in range(4):
        _cycle(s, torch, c3, mode)
