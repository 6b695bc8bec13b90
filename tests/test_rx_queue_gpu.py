"""The subframe batch queue (include/srsgpu/rx_queue.h), driven the way srsUE's PHY workers would
drive it (srsue/src/phy/phch_worker.cc:548-806, one subframe per worker call, several workers):
four threads each decode their own time-domain subframes through srsgpu_rxq_decode, the queue's
dispatcher batches them, and every TB must equal what the direct batch API (ofdm -> chest ->
pdsch_decode_dev in one call, tests/test_pipeline_gpu.py's chain) returns for the same subframes:
return codes, nof_iterations, data bytes — and the transmitted bytes at high SNR."""
import threading

import numpy as np
import pytest

from srsgpu_testlib import DlschOracle, PdschOracle
from test_pipeline_gpu import build_subframe

pytestmark = pytest.mark.gpu


def _direct(s, torch, xs, sfs, nof_prb, cell_id, N, tbs):
    n, gsz = len(xs), 14 * 12 * nof_prb
    ofdm = s.OfdmRx(nof_prb, N)
    chest = s.Chest(nof_prb, cell_id, max_grids=n)
    pd = s.Pdsch(nof_prb, cell_id, nof_softbuffers=n, max_sf=n)
    d_x = torch.from_numpy(np.stack(xs).reshape(-1)).cuda()
    d_grid = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    d_ce = torch.zeros_like(d_grid)
    d_noise = torch.zeros(n, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    assert ofdm.rx_dev(n, d_x.data_ptr(), 15 * N, d_grid.data_ptr(), gsz) == 0
    assert chest.estimate_dev([sf for sf, _ in sfs], d_grid.data_ptr(), gsz, d_ce.data_ptr(),
                              d_noise.data_ptr()) == 0
    pd.set_noise_dev(d_noise.data_ptr())
    dlen = tbs // 8 + 6
    sfl = []
    for i, (sf_idx, nre) in enumerate(sfs):
        pd.reset_softbuffer(i)
        sfl.append(s.make_sf(sf_idx=sf_idx, lstart=1, nof_prb=nof_prb, mod=3, nof_re=nre, rnti=1234,
                             tbs=tbs, softbuffer=i, grid_offset=i * gsz, data_offset=i * dlen))
    d_data = torch.zeros(n * dlen, dtype=torch.uint8, device="cuda")
    d_ret = torch.full((n,), 9, dtype=torch.int32, device="cuda")
    d_noi = torch.zeros(n, dtype=torch.int32, device="cuda")
    assert pd.decode_dev(sfl, d_grid.data_ptr(), d_ce.data_ptr(), gsz, d_data.data_ptr(), 8,
                         d_ret.data_ptr(), d_noi.data_ptr()) == 0
    torch.cuda.synchronize()
    out = (d_ret.cpu().numpy(), d_noi.cpu().numpy(), d_data.cpu().numpy().reshape(n, dlen),
           d_noise.cpu().numpy())
    for h in (pd, chest, ofdm):
        h.close()
    return out


def test_worker_threads_through_the_queue(oracle):
    import torch
    import srsgpu_phy as s
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(77)
    nof_prb, cell_id, tbs = 50, 3, 36696  # 10 MHz, MCS 28
    N = s.symbol_sz(nof_prb, True)
    n, nthreads = 24, 4
    xs, datas, sfs = [], [], []
    for i in range(n):
        sf_idx = [1, 2, 3, 4, 6, 7, 8, 9][i % 8]
        snr = 30.0 if i % 3 else 14.0  # some TBs fail, some need more half-iterations
        x, data, idx = build_subframe(po, dl, rng, nof_prb, cell_id, N, sf_idx, tbs, 1234, snr,
                                      rng.uniform(0, 6.28))
        xs.append(x)
        datas.append(data)
        sfs.append((sf_idx, idx.size))
    ret_d, noi_d, data_d, noise_d = _direct(s, torch, xs, sfs, nof_prb, cell_id, N, tbs)

    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=n, max_batch=8, max_wait_us=3000)
    dlen = tbs // 8 + 6
    outs = [np.zeros(dlen, np.uint8) for _ in range(n)]
    items = [q.item([xs[i]], s.make_sf(sf_idx=sfs[i][0], lstart=1, nof_prb=nof_prb, mod=3,
                                        nof_re=sfs[i][1], rnti=1234, tbs=tbs, softbuffer=i),
                    [outs[i]]) for i in range(n)]
    rcs = [None] * n

    def worker(w):
        for i in range(w, n, nthreads):
            rcs[i] = q.decode(items[i])

    th = [threading.Thread(target=worker, args=(w,)) for w in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    batches, done = q.stats()
    assert rcs == [0] * n and done == n
    assert batches < n  # the dispatcher batched the workers' subframes
    nb = (tbs + 24) // 8
    for i in range(n):
        assert items[i].ret[0] == ret_d[i] and items[i].noi[0] == noi_d[i], i
        assert (outs[i][:nb] == data_d[i][:nb]).all(), i
        assert abs(items[i].noise - noise_d[i]) <= 1e-6 * max(1.0, abs(noise_d[i])), i
        if i % 3:
            assert items[i].ret[0] == 0 and (outs[i][:tbs // 8] == datas[i]).all(), i
    # asynchronous form: submit everything, flush, then wait
    for i in range(n):
        items[i].reset_softbuffer[0] = 1
    tickets = [q.submit(items[i]) for i in range(n)]
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    assert all(items[i].ret[0] == ret_d[i] for i in range(n))
    # native worker pool (srsgpu_rxq_drive): 3 threads, every item submitted twice in a row of
    # 2n where item j + n reuses item j's softbuffer and output, so its submission must wait
    for i in range(n):
        items[i].ret[0] = 9
        outs[i][:] = 0
    t_sub, t_done, status = q.drive(items + items, 3, reuse=n)
    assert (status == 0).all() and (t_done >= t_sub).all()
    assert (t_sub[n:] >= t_done[:n]).all()  # reuse: the second round waited for the first
    for i in range(n):
        assert items[i].ret[0] == ret_d[i] and items[i].noi[0] == noi_d[i], i
        assert (outs[i][:nb] == data_d[i][:nb]).all(), i
    q.close()


def test_registered_outputs_written_in_place(oracle):
    """TB outputs that lie in a registered host block are written by the decoder itself over PCIe
    (no staging in the queue): the bytes, return codes and nof_iterations equal the direct batch API's;
    outputs outside the block (every third item) take the staged copy-back in the same batches; several
    batches in flight (three slots) keep every item's results its own"""
    import torch
    import srsgpu_phy as s
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(5)
    nof_prb, cell_id, tbs = 25, 9, 18336  # 5 MHz, MCS 28
    N = s.symbol_sz(nof_prb, True)
    n = 30
    xs, datas, sfs = [], [], []
    for i in range(n):
        sf_idx = [1, 2, 3, 4, 6, 7, 8, 9][i % 8]
        x, data, idx = build_subframe(po, dl, rng, nof_prb, cell_id, N, sf_idx, tbs, 1234, 30.0 if i % 4 else 12.0,
                                      rng.uniform(0, 6.28))
        xs.append(x)
        datas.append(data)
        sfs.append((sf_idx, idx.size))
    ret_d, noi_d, data_d, _ = _direct(s, torch, xs, sfs, nof_prb, cell_id, N, tbs)
    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=n, max_batch=4, max_wait_us=2000)
    dlen = tbs // 8 + 6
    block = np.zeros((n, dlen + 3), np.uint8)  # rows at odd offsets: no alignment needed
    q.register(block)
    own = [np.zeros(dlen, np.uint8) for _ in range(n)]
    outs = [own[i] if i % 3 == 0 else block[i, 3:3 + dlen] for i in range(n)]
    items = [q.item([xs[i]], s.make_sf(sf_idx=sfs[i][0], lstart=1, nof_prb=nof_prb, mod=3, nof_re=sfs[i][1],
                                        rnti=1234, tbs=tbs, softbuffer=i), [outs[i]]) for i in range(n)]
    tickets = [q.submit(it) for it in items]
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    nb = (tbs + 24) // 8
    for i in range(n):
        assert items[i].ret[0] == ret_d[i] and items[i].noi[0] == noi_d[i], i
        assert (outs[i][:nb] == data_d[i][:nb]).all(), i
    assert sum(int(items[i].ret[0] == 0) for i in range(n)) >= n // 2
    q.unregister(block)
    q.close()


def test_empty_noise_carried_across_batches(oracle):
    """EMPTY noise (srsUE's snr_estim_alg=empty, phch_worker.cc:557-564): only subframes 0 and 5
    estimate the noise (chest_dl.c:628-637); every other subframe keeps the latest estimate of an
    earlier subframe — across the queue's batch boundaries too, and 0 before any estimate
    (srslte_chest_dl_init). The queue's per-subframe noise must follow that order exactly."""
    import torch
    import srsgpu_phy as s
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(5)
    nof_prb, cell_id, tbs = 25, 11, 2216
    N = s.symbol_sz(nof_prb, True)
    order = [1, 2, 3, 0, 1, 4, 6, 5, 7, 8, 9, 1, 2, 0, 3]  # batches of 4 split the carries
    xs, sfs = [], []
    for sf_idx in order:
        x, _, idx = build_subframe(po, dl, rng, nof_prb, cell_id, N, sf_idx, tbs, 1234, 12.0,
                                   rng.uniform(0, 6.28))
        xs.append(x)
        sfs.append((sf_idx, idx.size))
    # the estimates of the 0 / 5 subframes, from the direct chest with the same settings
    n, gsz = len(xs), 14 * 12 * nof_prb
    ofdm = s.OfdmRx(nof_prb, N)
    chest = s.Chest(nof_prb, cell_id, max_grids=n)
    chest.set_cfg(noise_alg=2)
    d_x = torch.from_numpy(np.stack(xs).reshape(-1)).cuda()
    d_grid = torch.zeros(n * gsz, dtype=torch.complex64, device="cuda")
    d_ce = torch.zeros_like(d_grid)
    d_noise = torch.full((n,), -1.0, dtype=torch.float32, device="cuda")
    assert ofdm.rx_dev(n, d_x.data_ptr(), 15 * N, d_grid.data_ptr(), gsz) == 0
    assert chest.estimate_dev(order, d_grid.data_ptr(), gsz, d_ce.data_ptr(), d_noise.data_ptr()) == 0
    est = d_noise.cpu().numpy()
    expect, last = [], 0.0
    for i, sf_idx in enumerate(order):
        if sf_idx in (0, 5):
            assert est[i] > 0
            last = float(est[i])
        expect.append(last)
    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=n, max_batch=4, max_wait_us=200000)
    q.set_chest_cfg(noise_alg=2)
    outs = [np.zeros(tbs // 8 + 6, np.uint8) for _ in range(n)]
    items = [q.item([xs[i]], s.make_sf(sf_idx=sfs[i][0], lstart=1, nof_prb=nof_prb, mod=3,
                                        nof_re=sfs[i][1], rnti=1234, tbs=tbs, softbuffer=i),
                    [outs[i]]) for i in range(n)]
    tickets = [q.submit(it) for it in items]
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    got = [it.noise for it in items]
    assert np.allclose(got, expect, rtol=1e-6, atol=0), (got, expect)
    batches, done = q.stats()
    assert done == n and batches >= 4
    for h in (q, chest, ofdm):
        h.close()


def _queue_case(oracle, n=12, seed=41):
    import srsgpu_phy as s
    po, dl = PdschOracle(oracle), DlschOracle(oracle)
    rng = np.random.default_rng(seed)
    nof_prb, cell_id, tbs = 25, 7, 18336  # 5 MHz, MCS 28
    N = s.symbol_sz(nof_prb, True)
    xs, datas, sfs = [], [], []
    for i in range(n):
        sf_idx = [1, 2, 3, 4, 6, 7, 8, 9][i % 8]
        x, data, idx = build_subframe(po, dl, rng, nof_prb, cell_id, N, sf_idx, tbs, 1234, 30.0,
                                      rng.uniform(0, 6.28))
        xs.append(x)
        datas.append(data)
        sfs.append((sf_idx, idx.size))
    return nof_prb, cell_id, tbs, N, xs, datas, sfs


def _run_queue(s, q, xs, sfs, nof_prb, tbs):
    n = len(xs)
    outs = [np.zeros(tbs // 8 + 6, np.uint8) for _ in range(n)]
    items = [q.item([xs[i]], s.make_sf(sf_idx=sfs[i][0], lstart=1, nof_prb=nof_prb, mod=3,
                                        nof_re=sfs[i][1], rnti=1234, tbs=tbs, softbuffer=i),
                    [outs[i]]) for i in range(n)]
    tickets = [q.submit(it) for it in items]
    q.flush()
    assert all(q.wait(t) == 0 for t in tickets)
    return [it.ret[0] for it in items], [it.noi[0] for it in items], [it.noise for it in items], outs


@pytest.mark.parametrize("ingest", ["dma", "kernel"])
def test_registered_and_sc16_ingest(oracle, ingest, monkeypatch):
    """Zero-copy ingest (srsgpu_rxq_register: registered samples are DMA'd straight from the caller's
    pinned memory, runs of address-contiguous subframes one copy each — or, SRSGPU_RXQ_INGEST=kernel,
    read in place by the batch's ingest kernel) and SC16 input (int16 I/Q converted on the GPU): the
    same TBs, iterations and noise estimates, bit for bit, as the staged complex-float path on the same
    sample values — with registered and staged subframes mixed in one batch, registered subframes out
    of address order and handed over twice, and misaligned pointers falling back to staging."""
    import torch
    import srsgpu_phy as s
    monkeypatch.setenv("SRSGPU_RXQ_INGEST", ingest)
    nof_prb, cell_id, tbs, N, xs, datas, sfs = _queue_case(oracle)
    n = len(xs)
    # the radio's int16 samples and their float values (what a staged cf32 caller would hand over)
    scale = float(max(np.abs(x.view(np.float32)).max() for x in xs)) / 30000.0
    sc = [np.round(x.view(np.float32) / scale).astype(np.int16) for x in xs]
    xq = [(v.astype(np.float32) * np.float32(scale)).view(np.complex64) for v in sc]
    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=n, max_batch=n, max_wait_us=200000)
    want = _run_queue(s, q, xq, sfs, nof_prb, tbs)  # staged cf32
    assert q.ingest_stats() == (0, n)
    assert all(r == 0 for r in want[0])
    for i in range(n):
        assert (want[3][i][:tbs // 8] == datas[i]).all(), i
    # registered cf32: every other subframe lies in the registered block
    block = np.stack(xq[::2])
    q.register(block)
    mixed = [block[i // 2] if i % 2 == 0 else xq[i] for i in range(n)]
    got = _run_queue(s, q, mixed, sfs, nof_prb, tbs)
    assert got[:3] == want[:3] and all((a == b).all() for a, b in zip(got[3], want[3]))
    assert q.ingest_stats() == ((n + 1) // 2, n + n // 2)
    # a td pointer that is not 16-byte aligned is staged
    raw = np.zeros(block.nbytes + 16, np.uint8)
    q.register(raw)
    mis = raw[8:8 + xq[0].nbytes].view(np.complex64)
    mis[:] = xq[0]
    got1 = _run_queue(s, q, [mis] + xq[1:], sfs, nof_prb, tbs)
    assert got1[:3] == want[:3]
    z0, s0 = q.ingest_stats()
    assert (z0, s0) == ((n + 1) // 2, n + n // 2 + n)
    q.unregister(raw)
    q.unregister(block)
    # SC16: staged, then registered
    q.set_input_format(q.SC16, scale)
    got = _run_queue(s, q, sc, sfs, nof_prb, tbs)
    assert got[:3] == want[:3] and all((a == b).all() for a, b in zip(got[3], want[3]))
    blk16 = np.stack(sc)
    q.register(blk16)
    got = _run_queue(s, q, list(blk16), sfs, nof_prb, tbs)
    assert got[:3] == want[:3] and all((a == b).all() for a, b in zip(got[3], want[3]))
    assert q.ingest_stats()[0] == z0 + n
    # out of address order, one subframe twice in the batch
    perm = [5, 0, 0, 11, 3, 2, 1, 4, 10, 9, 7, 6][:n]
    got = _run_queue(s, q, [blk16[p] for p in perm], [sfs[p] for p in perm], nof_prb, tbs)
    for i, p in enumerate(perm):
        assert (got[0][i], got[1][i], got[2][i]) == (want[0][p], want[1][p], want[2][p]), i
        assert (got[3][i] == want[3][p]).all(), i

    def same(got):
        return got[:3] == want[:3] and all((a == b).all() for a, b in zip(got[3], want[3]))

    # rows a short gap apart in one registered region share one DMA span, the gap's bytes (other
    # samples) copied with them; rows alternating between two registered regions never share one
    junk = np.random.default_rng(5).integers(-30000, 30000, size=blk16.shape, dtype=np.int16)
    gap16 = np.empty((2 * n,) + blk16.shape[1:], np.int16)
    gap16[0::2] = blk16
    gap16[1::2] = junk
    q.register(gap16)
    assert same(_run_queue(s, q, list(gap16[0::2]), sfs, nof_prb, tbs))
    blk16b = blk16.copy()
    q.register(blk16b)
    assert same(_run_queue(s, q, [blk16[i] if i % 2 else blk16b[i] for i in range(n)], sfs, nof_prb, tbs))
    q.unregister(blk16b)
    q.unregister(gap16)
    q.unregister(blk16)
    # cf32 rows a gap apart in a full batch: the queue's DMA target holds exactly max_batch rows, so a
    # span bridges gaps only while the rows after it still fit
    q.set_input_format(q.CF32)
    gapf = np.empty((2 * n,) + xq[0].shape, np.complex64)
    gapf[0::2] = np.stack(xq)
    gapf[1::2] = np.random.default_rng(6).standard_normal((n, 2 * xq[0].size)).astype(np.float32).view(np.complex64)
    q.register(gapf)
    assert same(_run_queue(s, q, list(gapf[0::2]), sfs, nof_prb, tbs))
    q.unregister(gapf)
    q.close()
    torch.cuda.synchronize()


def test_paced_streams(oracle):
    """srsgpu_rxq_drive_paced: 6 streams, one subframe each per 1 ms tick for 40 ticks, 3 HARQ slots
    per stream, registered samples: every submission is decoded (acked, the transmitted bytes) and
    latencies are measured from the tick."""
    import srsgpu_phy as s
    nof_prb, cell_id, tbs, N, xs, datas, sfs = _queue_case(oracle, n=6, seed=43)
    streams, depth, ticks = 6, 3, 40
    q = s.RxQueue(nof_prb, cell_id, N, nof_softbuffers=streams * depth, max_batch=streams, max_wait_us=500)
    block = np.stack(xs)
    q.register(block)
    outs = [np.zeros(tbs // 8 + 6, np.uint8) for _ in range(streams * depth)]
    items = []
    for d in range(depth):
        for st in range(streams):
            k = d * streams + st
            items.append(q.item([block[st]], s.make_sf(sf_idx=sfs[st][0], lstart=1, nof_prb=nof_prb, mod=3,
                                                       nof_re=sfs[st][1], rnti=1234, tbs=tbs, softbuffer=k),
                                [outs[k]]))
    lat, status, acked, late = q.drive_paced(items, streams, depth, ticks, 1000, workers=2)
    assert (status == 0).all() and acked == streams * ticks
    assert (lat > 0).all() and np.isfinite(lat).all()
    for k in range(streams * depth):
        assert (outs[k][:tbs // 8] == datas[k % streams]).all(), k
    assert q.ingest_stats()[0] == streams * ticks
    q.close()
