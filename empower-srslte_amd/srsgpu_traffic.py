"""Mixed-bandwidth multi-cell downlink traffic on one GPU (BASELINE configs[4]).

Cells of {6, 25, 50, 100} PRB (1.4 / 5 / 10 / 20 MHz) each carry a share of the subframes,
interleaved round-robin. Every subframe holds one SISO PDSCH transport block with a random
allocation of 1..nof_prb PRB from PRB 0 and a random MCS 0..28 (TBS and modulation from the
36.213 tables, passed in as `table`), so code block sizes range over K = 40 .. 6144.

Transmit side (untimed, all on the GPU): DL-SCH + PDSCH encoding (srsgpu_pdsch_encode_dev), CRS
(srsgpu_chest_put_crs_dev), OFDM TX, AWGN.

Receive step (the hot path): per cell, the front end runs as one batch over that cell's
subframes — OFDM FFT, CRS channel estimation, PDSCH LLRs (RE extraction, MMSE with the device
noise estimate, demapping, descrambling) into one shared LLR buffer. Then ONE DL-SCH call decodes
the transport blocks of all cells together (srsgpu_dlsch_decode_dev): the engine bins the code
blocks by decoder variant and size on the device side, so mixed K costs no per-cell launches.
Reference flow per subframe: srslte_ofdm_rx_sf -> srslte_chest_dl_estimate -> srslte_pdsch_decode
(lib/src/phy/ue/ue_dl.c:379-433,580).
"""
import ctypes
import time

import numpy as np

import srsgpu_phy as s

BITS_PER_SYMBOL = {1: 2, 2: 4, 3: 6}
MAX_CODE_RATE = 0.93  # 36.213 7.1.7: a UE may skip TBs above this effective rate


def plan(table, n_sf, prbs=(6, 25, 50, 100), seed=5, mcs=None, full_band=False):
    """The subframes of one traffic job, deterministic in its arguments (every rank of a sharded
    job draws the same plan): subframe i belongs to the cell of prbs[i % len(prbs)] and carries one
    TB with a random allocation of L PRB from PRB 0 and a random MCS (or the pinned ones), redrawn
    while the code rate exceeds MAX_CODE_RATE. Returns dicts {sf, prb, cell, L, mcs, mod, tbs, nre,
    sf_idx, lstart} in subframe order."""
    rng = np.random.default_rng(seed)
    mods, tbs_tab = table["mod_by_mcs"], table["tbs_by_prb_mcs"]
    out = [None] * n_sf
    for ci, prb in enumerate(prbs):
        cell = s.srsgpu_cell_t(prb, 1 + ci, 1, 1)
        lstart = 2 if prb <= 10 else 1
        for j, i in enumerate(i for i in range(n_sf) if i % len(prbs) == ci):
            sfi = 1 + (j % 4)
            while True:
                L = prb if full_band else int(rng.integers(1, prb + 1))
                m = mcs if mcs is not None else int(rng.integers(0, 29))
                mod, tbs = mods[m], tbs_tab[L - 1][m]
                mask = np.zeros((2, prb), np.uint8)
                mask[:, :L] = 1
                probe = s.make_sf(sf_idx=sfi, lstart=lstart, prb=mask, nof_prb=prb, mod=mod)
                nre = s._lib.srsgpu_pdsch_nof_re(ctypes.byref(cell), ctypes.byref(probe))
                if (tbs + 24) <= MAX_CODE_RATE * nre * BITS_PER_SYMBOL[mod] or mcs is not None:
                    break
            out[i] = {"sf": i, "prb": prb, "cell": ci, "L": L, "mcs": m, "mod": mod, "tbs": tbs,
                      "nre": nre, "sf_idx": sfi, "lstart": lstart}
    return out


def tb_weights(table, sf_plan, max_halfits=8):
    """decoding cost per planned subframe (sum of K of its TB's code blocks x the budget), the
    weights of the multi-GPU partition (srsgpu_shard.weighted)"""
    import srsgpu_shard as sh
    return [sh.tb_weight(table["cbsegm_C_C1_K1_C2_K2_F"][str(p["tbs"])], max_halfits) for p in sf_plan]


class MixedCells:
    def __init__(self, table, n_sf, torch, dev, prbs=(6, 25, 50, 100), seed=5, stream=None,
                 snr_db=30.0, max_halfits=8, mcs=None, full_band=False, keep=None, standard_rate=True,
                 early_stop=True, ce_rows=True, rotate=1, engines=1, tail_stream=None, fe_stream=None):
        """n_sf subframes round-robin over the cells of `prbs`; mcs / full_band pin the MCS and
        the allocation (e.g. prbs=(100,), mcs=28, full_band=True is the C3 subframe as coded
        traffic). keep: the subframe indices this instance builds and receives (a rank's shard
        of one planned job, srsgpu_shard); default all. standard_rate: the 3GPP FFT sizes (2048 at
        20 MHz) or srsLTE's reduced ones (1536, srslte_symbol_sz without standard rates).
        early_stop False: every code block runs max_halfits (srsgpu_dlsch_set_early_stop).
        ce_rows: the estimator hands the PDSCH stage its compact rows (srsgpu_chest_set_ce_rows /
        srsgpu_pdsch_set_ce_rows: identical LLRs, 3.5x fewer estimate bytes).
        rotate R > 1: R descriptor sets that differ in their softbuffers (set r uses softbuffers
        r * ntb ..), used in turn by successive steps, so no two consecutive calls of the PDSCH and
        DL-SCH stages repeat their inputs and their repeat-call caches never hit, as for a receiver
        whose grants change every subframe.
        engines 2 with tail_stream (a HIP stream handle): two DL-SCH engines (each with its own LLR,
        output and softbuffer sets) used by alternate steps, each decoding its early-stop tail on
        tail_stream (srsgpu_dlsch_set_tail_stream): a step's front end and first half-iteration run
        while the previous step's few straggling code blocks finish beside them. The attributes dlsch,
        d_e, d_data, d_ret, d_noi name the engine of the last step.
        fe_stream (with engines 2 and tail_stream): the front end (OFDM, estimator, PDSCH LLRs) on a
        stream of its own, so a batch's front end runs beside the previous batch's decoder; it starts
        once the LLR buffer it writes is free (the tail of that engine's previous call, an event on the
        tail stream) and the DL-SCH call waits for it (an event on fe_stream)."""
        self.torch, self.dev = torch, dev
        self._split = bool(fe_stream) and bool(tail_stream) and int(engines) > 1
        if self._split:
            self._fe = torch.cuda.ExternalStream(fe_stream, device=dev)
            self._ln = torch.cuda.ExternalStream(stream, device=dev) if stream else torch.cuda.current_stream(dev)
            self._tl = torch.cuda.ExternalStream(tail_stream, device=dev)
            self._ev_fe = torch.cuda.Event()
            self._ev_tail = [None, None]
        fe_st = fe_stream if self._split else stream
        self.max_halfits = max_halfits
        sf_plan = plan(table, n_sf, prbs, seed, mcs, full_band)
        keep = set(range(n_sf)) if keep is None else set(int(k) for k in keep)
        self.kept = sorted(keep)
        self.rotate, self.cur = max(1, int(rotate)), 0
        self.host_s = [0.0, 0.0]
        self.cells = []
        self.sf_total = len(self.kept)
        e_off = d_off = 0
        tb_list = []
        for ci, prb in enumerate(prbs):
            mine = [p for p in sf_plan if p["cell"] == ci and p["sf"] in keep]
            n = len(mine)
            if n == 0:
                continue
            N = s.symbol_sz(prb, standard_rate)
            gsz = 14 * 12 * prb
            c = {"prb": prb, "N": N, "gsz": gsz, "n": n, "id": 1 + ci,
                 "lstart": 2 if prb <= 10 else 1}
            c["ofdm"] = s.OfdmRx(prb, N, stream=fe_st)
            c["chest"] = s.Chest(prb, c["id"], max_grids=n, stream=fe_st)
            c["pd"] = s.Pdsch(prb, c["id"], nof_softbuffers=1, max_cb=13, max_sf=n, stream=fe_st)
            c["chest"].set_ce_rows(ce_rows)
            c["pd"].set_ce_rows(4 if ce_rows else 0)
            sfs, e_offs, sf_idx = [], [], []
            for j, p in enumerate(mine):
                mask = np.zeros((2, prb), np.uint8)
                mask[:, :p["L"]] = 1
                qm = BITS_PER_SYMBOL[p["mod"]]
                sf = s.make_sf(sf_idx=p["sf_idx"], lstart=p["lstart"], prb=mask, nof_prb=prb, mod=p["mod"],
                               nof_re=p["nre"], rnti=1234, tbs=p["tbs"], softbuffer=len(tb_list),
                               grid_offset=j * gsz, data_offset=d_off)
                sfs.append(sf)
                e_offs.append(e_off)
                sf_idx.append(p["sf_idx"])
                tb_list.append({"tbs": p["tbs"], "rv": 0, "Qm": qm, "nof_e_bits": p["nre"] * qm,
                                "softbuffer": len(tb_list), "e_offset": e_off, "data_offset": d_off,
                                "sf": p["sf"]})
                e_off += (p["nre"] * qm + 63) // 64 * 64
                d_off += s.dlsch_data_len(p["tbs"]) + 2
            # descriptor arrays built once (the receive step reuses them every batch)
            c.update(sfs=s.make_sf_array(sfs), e_offs=(ctypes.c_uint64 * n)(*e_offs),
                     sf_idx=(ctypes.c_uint32 * n)(*sf_idx))
            c["sfs_rot"] = [c["sfs"]]
            for r in range(1, self.rotate):
                arr = (s.srsgpu_pdsch_sf_t * n)(*sfs)
                for j in range(n):
                    arr[j].softbuffer[0] = sfs[j].softbuffer[0] + r * n_sf
                c["sfs_rot"].append(arr)
            self.cells.append(c)
        self.tb_list = tb_list
        self.tb_array = s.make_tb_array(tb_list)
        self.ntb = len(tb_list)
        self.tb_rot = [self.tb_array] + [
            s.make_tb_array([dict(t, softbuffer=t["softbuffer"] + r * self.ntb) for t in tb_list])
            for r in range(1, self.rotate)]
        self.ncb = sum(int(table["cbsegm_C_C1_K1_C2_K2_F"][str(t["tbs"])][0]) for t in tb_list)
        self.bits = sum(t["tbs"] for t in tb_list)
        self.nengine, self.eng = max(1, int(engines)), 0
        z = lambda n, dt: torch.zeros(n, dtype=dt, device=dev)  # noqa: E731
        self._dl, self._de, self._dd, self._dr, self._dn = [], [], [], [], []
        for _ in range(self.nengine):
            dl = s.Dlsch(max(self.ntb * self.rotate, 1), max_cb=13, max_cbs_per_call=max(self.ncb, 1), stream=stream)
            dl.set_early_stop(early_stop)
            if tail_stream and self.nengine > 1:
                dl.set_tail_stream(tail_stream)
            self._dl.append(dl)
            self._de.append(z(max(e_off, 1), torch.int16))
            self._dd.append(z(max(d_off, 1), torch.uint8))
            self._dr.append(z(self.ntb, torch.int32))
            self._dn.append(z(self.ntb, torch.int32))
        self.d_data_tx = torch.randint(0, 256, (max(d_off, 1),), dtype=torch.uint8, device=dev,
                                       generator=torch.Generator(device=dev).manual_seed(seed))
        for c in self.cells:
            n, gsz, N = c["n"], c["gsz"], c["N"]
            c["grid"] = z(n * gsz, torch.complex64)
            c["ce"] = z(n * gsz, torch.complex64)
            c["noise"] = z(n, torch.float32)
            c["x"] = z(n * 15 * N, torch.complex64)
            c["pd"].set_noise_dev(c["noise"].data_ptr())
        self._transmit(snr_db, seed)

    dlsch = property(lambda self: self._dl[self.eng])
    d_e = property(lambda self: self._de[self.eng])
    d_data = property(lambda self: self._dd[self.eng])
    d_ret = property(lambda self: self._dr[self.eng])
    d_noi = property(lambda self: self._dn[self.eng])

    def _transmit(self, snr_db, seed):
        torch = self.torch
        g = torch.Generator(device=self.dev).manual_seed(seed + 1)
        for c in self.cells:
            n, gsz, N = c["n"], c["gsz"], c["N"]
            grid = self.torch.zeros(n * gsz, dtype=torch.complex64, device=self.dev)
            assert c["pd"].encode_dev(c["sfs"], self.d_data_tx.data_ptr(), grid.data_ptr()) == 0
            assert c["chest"].put_crs_dev(c["sf_idx"], grid.data_ptr(), gsz) == 0
            assert c["ofdm"].tx_dev(n, grid.data_ptr(), gsz, c["x"].data_ptr(), 15 * N) == 0
            torch.cuda.synchronize(self.dev)
            p = c["x"].abs().pow(2).mean().item()
            sd = float(np.sqrt(p / 10 ** (snr_db / 10) / 2))
            c["x"] += (sd * torch.randn(c["x"].shape, dtype=torch.complex64, device=self.dev,
                                        generator=g)).to(torch.complex64)

    def front_end(self):
        """per cell: OFDM RX, channel estimation, PDSCH LLRs into the shared LLR buffer"""
        for c in self.cells:
            n, gsz, N = c["n"], c["gsz"], c["N"]
            assert c["ofdm"].rx_dev(n, c["x"].data_ptr(), 15 * N, c["grid"].data_ptr(), gsz) == 0
            assert c["chest"].estimate_dev(c["sf_idx"], c["grid"].data_ptr(), gsz, c["ce"].data_ptr(),
                                           c["noise"].data_ptr()) == 0
            assert c["pd"].llr_dev(c["sfs_rot"][self.cur], c["grid"].data_ptr(), c["ce"].data_ptr(), gsz,
                                   self.d_e.data_ptr(), c["e_offs"]) == 0

    def decode(self):
        """one DL-SCH call over every cell's transport blocks (new TBs: softbuffers reset)"""
        self.dlsch.reset_range(self.cur * self.ntb, self.ntb)
        assert self.dlsch.decode_dev(self.tb_rot[self.cur], self.d_e.data_ptr(), self.d_data.data_ptr(),
                                     self.max_halfits, self.d_ret.data_ptr(),
                                     self.d_noi.data_ptr()) == 0

    def step(self):
        """one receive batch; host_s accumulates the host (enqueue) seconds of the front end and of the
        DL-SCH call"""
        self.cur = (self.cur + 1) % self.rotate
        self.eng = (self.eng + 1) % self.nengine
        t0 = time.perf_counter()
        if self._split:
            ev = self._ev_tail[self.eng]
            if ev is not None:
                self._fe.wait_event(ev)  # the engine's previous tail has read its LLR buffer
            self.front_end()
            self._ev_fe.record(self._fe)
            self._ln.wait_event(self._ev_fe)
            t1 = time.perf_counter()
            self.decode()
            ev = self._ev_tail[self.eng] or self.torch.cuda.Event()
            ev.record(self._tl)  # everything of this call on the tail stream
            self._ev_tail[self.eng] = ev
            self.host_s[0] += t1 - t0
            self.host_s[1] += time.perf_counter() - t1
            return
        if self.nengine > 1:
            # the engine's previous call may still read its LLR buffer on the tail stream (the P1 loads,
            # the rows of failed TBs): the front end rewrites that buffer only after it
            self.dlsch.join_tail()
        self.front_end()
        t1 = time.perf_counter()
        self.decode()
        self.host_s[0] += t1 - t0
        self.host_s[1] += time.perf_counter() - t1

    def check(self):
        """(acked TBs, TBs whose bytes equal the transmitted ones, mean nof_iterations)"""
        ret = self.d_ret.cpu().numpy()
        tx = self.d_data_tx.cpu().numpy()
        rx = self.d_data.cpu().numpy()
        good = 0
        for t, r in zip(self.tb_list, ret):
            o, nb = t["data_offset"], t["tbs"] // 8
            good += int(r == 0 and (tx[o:o + nb] == rx[o:o + nb]).all())
        return int((ret == 0).sum()), good, float(self.d_noi.cpu().numpy().mean())

    def decoded_bits(self, table):
        """SURVEY §8(d)'s decoded bits of the last decode: the sum of K over the code blocks whose
        CRC passed. A TB that acks passed every code block; a failed TB contributes the code
        blocks its softbuffer marks in cb_crc (sch.c:394-401)."""
        ret = self.d_ret.cpu().numpy()
        seg = table["cbsegm_C_C1_K1_C2_K2_F"]
        total = 0
        for t, r in zip(self.tb_list, ret):
            C, _c1, K1, C2, K2, _f = seg[str(t["tbs"])]
            ks = [K2 if i < C2 else K1 for i in range(C)]
            if r == 0:
                total += sum(ks)
            else:
                crc = self.dlsch.read_cb_crc(self.softbuffer_of(t))
                total += sum(k for k, c in zip(ks, crc) if c)
        return total

    def softbuffer_of(self, t):
        """the softbuffer TB t used in the last step (descriptor set self.cur)"""
        return t["softbuffer"] + self.cur * self.ntb

    def close(self):
        for c in self.cells:
            for k in ("ofdm", "chest", "pd"):
                c[k].close()
        for dl in self._dl:
            dl.close()


class MimoSubframes:
    """Coded two-port subframes on one GPU (BASELINE configs[3] as real codewords): n subframes of a
    20 MHz cell with 2 CRS ports and 2 rx antennas, each carrying the full-band PDSCH of one MIMO type
    (default TM3 large-delay CDD with two MCS-28 TBs of TBS 75376, tb_cw_swap on odd subframes).

    Transmit side (untimed, on the GPU): srsgpu_pdsch_encode_ports_dev (DL-SCH encoding, per-codeword
    scrambling and modulation, CDD / transmit-diversity / codebook precoding into both ports' grids),
    the CRS of both ports (srsgpu_chest_put_crs_dev), OFDM TX per port, a 2x2 flat channel per
    subframe (well conditioned, random phases) and AWGN at snr_db.
    Receive step: OFDM FFT of both antennas, channel estimation of both ports on each antenna, PDSCH
    (2x2 MMSE for CDD / spatial multiplexing, SFBC for transmit diversity) and DL-SCH with CRC early
    stop, all through srsgpu_pdsch_decode_dev. keep: the subframe indices of a global job this instance
    handles (a rank's shard); subframe i's content depends only on i."""

    def __init__(self, torch, dev, n_sf, seed=31, stream=None, snr_db=30.0, mimo=None, mcs=28, nof_prb=100,
                 cell_id=1, keep=None, max_halfits=8, codebook=1, nof_tb=2, early_stop=True, ce_rows=True,
                 nof_ports=2, cp=0):
        import ctypes as ct
        self.torch, self.dev, self.max_halfits = torch, dev, max_halfits
        mimo = s.MIMO_CDD if mimo is None else mimo
        self.kept = sorted(set(range(n_sf)) if keep is None else set(int(k) for k in keep))
        n = len(self.kept)
        self.n = n
        self.nof_prb, self.cell_id = nof_prb, cell_id
        N = s.symbol_sz(nof_prb, True)
        self.N, gsz = N, (12 if cp else 14) * 12 * nof_prb  # extended CP (cp=1): 12 symbols
        self.gsz = gsz
        ntb = 1 if mimo in (s.MIMO_TX_DIVERSITY, s.MIMO_SINGLE_ANTENNA) else nof_tb
        self.ntb = ntb
        P = self.nports = nof_ports  # 4: transmit diversity over ports 0-3 (estimates in full grids)
        assert (P == 2 or (P == 4 and mimo == s.MIMO_TX_DIVERSITY and not ce_rows) or
                (P == 1 and mimo == s.MIMO_SINGLE_ANTENNA))
        assert not (cp and ce_rows)  # the 4 compact rows are the normal-CP CRS symbols
        tbs = s._lib.srsgpu_ra_tbs_from_idx(s._lib.srsgpu_ra_tbs_idx_from_mcs(mcs), nof_prb)
        mod = 1 if mcs < 10 else 2 if mcs < 17 else 3
        self.tbs = tbs
        self.ofdm = s.OfdmRx(nof_prb, N, stream=stream, cp=cp)
        self.chest = s.Chest(nof_prb, cell_id, max_grids=2 * n, stream=stream, nof_ports=P, cp=cp)
        self.pd = s.Pdsch(nof_prb, cell_id, nof_ports=P, nof_rx_ant=2, nof_softbuffers=2 * n, max_cb=13, max_sf=n,
                          stream=stream, cp=cp)
        s._lib.srsgpu_dlsch_set_early_stop(s._vp(self.pd.dlsch_q), int(bool(early_stop)))
        self.chest.set_ce_rows(ce_rows)  # compact estimate rows, identical LLRs (as MixedCells)
        self.pd.set_ce_rows(4 if ce_rows else 0)
        dlen = s.dlsch_data_len(tbs) + 2
        self.dlen = dlen
        sfs = []
        for j, i in enumerate(self.kept):
            sfi = 1 + (i % 4)
            sf = s.make_sf(sf_idx=sfi, lstart=1, nof_prb=nof_prb, mod=(mod, mod), rnti=1234,
                           tbs=(tbs, tbs if ntb == 2 else 0), softbuffer=(2 * j, 2 * j + 1), mimo=mimo,
                           grid_offset=j * 2 * gsz, ce_offset=j * 2 * P * gsz,
                           data_offset=(2 * j * dlen, (2 * j + 1) * dlen), tb_cw_swap=i % 2 if ntb == 2 else 0,
                           codebook_idx=codebook if mimo == s.MIMO_SPATIAL_MULTIPLEX else 0)
            sf.nof_re = self.pd.nof_re(sf)
            sfs.append(sf)
        self.sfs = s.make_sf_array(sfs)
        self.nre = sfs[0].nof_re
        # the transmitter's [sf][port] grids: P planes per subframe (the receive grids hold 2 rx antennas)
        for j, sf in enumerate(sfs):
            sf.grid_offset = j * P * gsz
        self.sfs_tx = s.make_sf_array(sfs)
        self.grid_sf = (ct.c_uint32 * (2 * n))(*[1 + (i % 4) for i in self.kept for _ in range(2)])  # [sf][rx]
        self.sf_list = (ct.c_uint32 * n)(*[1 + (i % 4) for i in self.kept])  # [sf]
        z = lambda k, dt: torch.zeros(k, dtype=dt, device=dev)  # noqa: E731
        # TB bytes: subframe i's content is a function of i (the same on every rank)
        g = torch.Generator(device="cpu").manual_seed(seed)
        base = torch.randint(0, 256, (16, 2, dlen), dtype=torch.uint8, generator=g)
        idx = torch.tensor([i % 16 for i in self.kept])
        self.d_data_tx = base[idx].reshape(-1).to(dev)
        self.d_data = z(2 * n * dlen, torch.uint8)
        self.d_ret = z(2 * n, torch.int32)
        self.d_noi = z(2 * n, torch.int32)
        self.grid = z(2 * n * gsz, torch.complex64)
        self.ce = z(2 * P * n * gsz, torch.complex64)
        self.noise = z(2 * P * n, torch.float32)
        self.x = z(2 * n * 15 * N, torch.complex64)
        self.pd.set_noise_dev(self.noise.data_ptr())
        self._transmit(snr_db, seed, stream)

    def _transmit(self, snr_db, seed, stream):
        torch, n, gsz, N, P = self.torch, self.n, self.gsz, self.N, self.nports
        txg = torch.zeros(P * n * gsz, dtype=torch.complex64, device=self.dev)  # [sf][port] grids
        assert self.pd.encode_dev((self.sfs_tx, n), self.d_data_tx.data_ptr(), txg.data_ptr(), port_stride=gsz) == 0
        # every port's CRS: grid i's port p at plane i * P + p, n grids (one per subframe)
        assert self.chest.put_crs_dev(self.sf_list, txg.data_ptr(), gsz) == 0
        xp = torch.zeros(P * n * 15 * N, dtype=torch.complex64, device=self.dev)
        assert self.ofdm.tx_dev(P * n, txg.data_ptr(), gsz, xp.data_ptr(), 15 * N) == 0
        torch.cuda.synchronize(self.dev)
        del txg
        xp = xp.reshape(n, P, 15 * N)
        # a flat 2 x P channel per subframe, from the subframe's global index
        g = torch.Generator(device="cpu").manual_seed(seed + 7)
        ph = torch.rand(16, 2, P, generator=g) * 6.283
        amp = {1: torch.tensor([[1.0], [0.45]]), 2: torch.tensor([[1.0, 0.45], [0.45, 1.0]]),
               4: torch.tensor([[1.0, 0.45, 0.8, 0.3], [0.45, 1.0, 0.3, 0.8]])}[P]
        H = (amp * torch.exp(1j * ph)).to(torch.complex64)
        Hs = H[torch.tensor([i % 16 for i in self.kept])].to(self.dev)  # [sf][rx][port]
        y = torch.einsum("sap,spt->sat", Hs, xp)
        del xp
        p = y.abs().pow(2).mean().item()
        sd = float(np.sqrt(p / 10 ** (snr_db / 10) / 2))
        gn = torch.Generator(device=self.dev).manual_seed(seed + 11)
        y += (sd * torch.randn(y.shape, dtype=torch.complex64, device=self.dev, generator=gn)).to(torch.complex64)
        self.x.copy_(y.reshape(-1))
        torch.cuda.synchronize(self.dev)

    def step(self):
        n, gsz, N = self.n, self.gsz, self.N
        self.pd.reset_softbuffer(0, 2 * n)  # new TBs
        assert self.ofdm.rx_dev(2 * n, self.x.data_ptr(), 15 * N, self.grid.data_ptr(), gsz) == 0
        assert self.chest.estimate_dev(self.grid_sf, self.grid.data_ptr(), gsz, self.ce.data_ptr(),
                                       self.noise.data_ptr()) == 0
        assert self.pd.decode_dev(self.sfs, self.grid.data_ptr(), self.ce.data_ptr(), gsz, self.d_data.data_ptr(),
                                  self.max_halfits, self.d_ret.data_ptr(), self.d_noi.data_ptr()) == 0

    def check(self):
        """(acked TBs, TBs whose bytes equal the transmitted ones, mean nof_iterations)"""
        ret = self.d_ret.cpu().numpy()[:self.ntb * self.n] if self.ntb == 2 else self.d_ret.cpu().numpy()[:self.n]
        tx, rx = self.d_data_tx.cpu().numpy(), self.d_data.cpu().numpy()
        good = 0
        nb = self.tbs // 8
        for k, r in enumerate(ret):
            j, t = (k // 2, k % 2) if self.ntb == 2 else (k, 0)
            o = (2 * j + t) * self.dlen
            good += int(r == 0 and (tx[o:o + nb] == rx[o:o + nb]).all())
        noi = self.d_noi.cpu().numpy()[:len(ret)]
        return int((ret == 0).sum()), good, float(noi.mean())

    def decoded_bits(self, table):
        """SURVEY §8(d)'s decoded bits of the last decode (as MixedCells.decoded_bits): the sum of K
        over the code blocks whose CRC passed, from the return codes and the softbuffers' cb_crc"""
        C, _c1, K1, C2, K2, _f = table["cbsegm_C_C1_K1_C2_K2_F"][str(self.tbs)]
        ret = self.d_ret.cpu().numpy()
        ks = [K2] * C2 + [K1] * (C - C2)  # the C2 smaller blocks first (36.212 5.1.2)
        total = 0
        for k in range(self.ntb * self.n):
            j, t = (k // 2, k % 2) if self.ntb == 2 else (k, 0)
            if ret[k] == 0:
                total += sum(ks)
            else:
                crc = self.pd.read_cb_crc(2 * j + t)
                total += sum(kk for kk, ok in zip(ks, crc[:C]) if ok)
        return total

    def close(self):
        for h in (self.ofdm, self.chest, self.pd):
            h.close()
