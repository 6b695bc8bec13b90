"""Test-side helpers: ctypes bindings for the CPU oracle (oracle/liboracle.so), the optional
reference build (oracle/_ref/libsrsref.so, this container only) and synthetic LLR generation.

TEST INFRASTRUCTURE ONLY — the product path (empower-srslte_amd) never imports this.
"""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libsrsref.so")

# srslte_tdec_impl_type_t (turbodecoder_impl.h:33-42)
AUTO, GENERIC, SSE, SSE_WINDOW, AVX_WINDOW, SSE8_WINDOW, AVX8_WINDOW = 0, 1, 2, 3, 4, 5, 6
CRC24A, CRC24B = 0x1864CFB, 0x1800063

_i16p = ctypes.POINTER(ctypes.c_int16)
_i8p = ctypes.POINTER(ctypes.c_int8)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u16p = ctypes.POINTER(ctypes.c_uint16)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


class _Lib:
    def __init__(self, path, prefix):
        self.lib = ctypes.CDLL(path)
        self.p = prefix
        f = self._f
        f("tdec_run").argtypes = [ctypes.c_int, ctypes.c_int, _i16p, ctypes.c_uint32,
                                  ctypes.c_uint32, _u8p, _i16p, _i16p]
        f("tdec_run").restype = ctypes.c_int
        f("interl").argtypes = [ctypes.c_uint32, ctypes.c_uint32, _u16p, _u16p]
        f("tcod_encode").argtypes = [_u8p, _u8p, ctypes.c_uint32]
        f("crc_checksum_byte").argtypes = [ctypes.c_uint32, ctypes.c_int, _u8p, ctypes.c_uint32]
        f("crc_checksum_byte").restype = ctypes.c_uint32

    def _f(self, name):
        return getattr(self.lib, self.p + name)

    def tdec_run(self, impl, sb_layout, inp, K, nhalf):
        inp = np.ascontiguousarray(inp, dtype=np.int16)
        dec = np.zeros((nhalf, K // 8), np.uint8)
        app1 = np.zeros(K, np.int16)
        ext1 = np.zeros(K, np.int16)
        r = self._f("tdec_run")(impl, sb_layout, _ptr(inp, _i16p), K, nhalf, _ptr(dec, _u8p),
                                _ptr(app1, _i16p), _ptr(ext1, _i16p))
        assert r == 0, r
        return dec, app1, ext1

    def interl(self, K, nsb):
        f = np.zeros(K, np.uint16)
        r = np.zeros(K, np.uint16)
        assert self._f("interl")(K, nsb, _ptr(f, _u16p), _ptr(r, _u16p)) == 0
        return f, r

    def tcod_encode(self, bits):
        bits = np.ascontiguousarray(bits, dtype=np.uint8)
        K = bits.size
        out = np.zeros(3 * K + 12, np.uint8)
        assert self._f("tcod_encode")(_ptr(bits, _u8p), _ptr(out, _u8p), K) == 0
        return out

    def crc(self, poly, data, len_bits, order=24):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        return self._f("crc_checksum_byte")(poly, order, _ptr(data, _u8p), len_bits)


class Oracle(_Lib):
    def __init__(self):
        super().__init__(ORACLE_SO, "orc_")
        L = self.lib
        L.orc_tdec8_run.argtypes = [ctypes.c_int, ctypes.c_int, _i8p, ctypes.c_uint32,
                                    ctypes.c_uint32, _u8p]
        L.orc_tdec8_run16.argtypes = [ctypes.c_int, _i16p, ctypes.c_uint32, ctypes.c_uint32, _u8p]
        L.orc_tdec_input_len.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32]
        L.orc_tdec_decode_cb.argtypes = [ctypes.c_int, ctypes.c_int, _i16p, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u8p,
                                         _u32p]
        L.orc_cbsegm.argtypes = [ctypes.c_uint32] + [_u32p] * 6

    def input_len(self, impl, sb, K):
        return self.lib.orc_tdec_input_len(impl, sb, K)

    def tdec8_run(self, impl, sb_layout, inp, K, nhalf):
        """8-bit path (srslte_tdec_iteration_8bit); decisions per half-iteration, or None where
        the reference has no defined result (orc_tdec8_run returns -2)"""
        inp = np.ascontiguousarray(inp, dtype=np.int8)
        dec = np.zeros((nhalf, K // 8), np.uint8)
        r = self.lib.orc_tdec8_run(impl, sb_layout, _ptr(inp, _i8p), K, nhalf, _ptr(dec, _u8p))
        if r == -2:
            return None
        assert r == 0, r
        return dec

    def tdec8_run16(self, impl, inp, K, nhalf):
        inp = np.ascontiguousarray(inp, dtype=np.int16)
        dec = np.zeros((nhalf, K // 8), np.uint8)
        assert self.lib.orc_tdec8_run16(impl, _ptr(inp, _i16p), K, nhalf, _ptr(dec, _u8p)) == 0
        return dec

    def decode_cb(self, impl, sb, inp, K, max_halfits, poly, crc_len):
        inp = np.ascontiguousarray(inp, dtype=np.int16)
        out = np.zeros(K // 8, np.uint8)
        noi = ctypes.c_uint32(0)
        ok = self.lib.orc_tdec_decode_cb(impl, sb, _ptr(inp, _i16p), K, max_halfits, poly,
                                         crc_len, _ptr(out, _u8p), ctypes.byref(noi))
        return ok, out, noi.value

    def cbsegm(self, tbs):
        v = [ctypes.c_uint32(0) for _ in range(6)]
        assert self.lib.orc_cbsegm(tbs, *[ctypes.byref(x) for x in v]) == 0
        return tuple(x.value for x in v)


class OrcSoftbuffer(ctypes.Structure):
    _fields_ = [("max_cb", ctypes.c_uint32), ("buffer", _i16p), ("data", _u8p),
                ("cb_crc", _u8p), ("tb_crc", ctypes.c_uint8)]


SOFTBUFFER_SIZE = 18600


class DlschOracle:
    """Bindings of oracle/dlsch_oracle.c (rate matching, TB encode/decode with softbuffer)."""

    def __init__(self, oracle):
        L = self.lib = oracle.lib
        u32 = ctypes.c_uint32
        L.orc_rm_turbo_rx_table.argtypes = [u32, u32, u32, _u16p]
        L.orc_rm_turbo_rx.argtypes = [_i16p, _i16p, u32, u32, u32, u32]
        L.orc_rm_turbo_tx.argtypes = [_u8p, u32, u32, _u8p, u32]
        L.orc_dlsch_encode.argtypes = [u32, u32, u32, u32, _u8p, _u8p]
        L.orc_softbuffer_init.argtypes = [ctypes.POINTER(OrcSoftbuffer), u32]
        L.orc_softbuffer_reset.argtypes = [ctypes.POINTER(OrcSoftbuffer)]
        L.orc_softbuffer_free.argtypes = [ctypes.POINTER(OrcSoftbuffer)]
        L.orc_dlsch_decode.argtypes = [ctypes.POINTER(OrcSoftbuffer), u32, u32, u32, u32, _i16p,
                                       _u8p, u32, _u32p]

    def rx_table(self, K, rv, nsb):
        t = np.zeros(3 * K + 12, np.uint16)
        assert self.lib.orc_rm_turbo_rx_table(K, rv, nsb, _ptr(t, _u16p)) == 0
        return t

    def rm_rx(self, e, out, K, rv, nsb):
        e = np.ascontiguousarray(e, np.int16)
        assert self.lib.orc_rm_turbo_rx(_ptr(e, _i16p), _ptr(out, _i16p), e.size, K, rv, nsb) == 0
        return out

    def rm_tx(self, coded, K, rv, E):
        coded = np.ascontiguousarray(coded, np.uint8)
        e = np.zeros(E, np.uint8)
        assert self.lib.orc_rm_turbo_tx(_ptr(coded, _u8p), K, rv, _ptr(e, _u8p), E) == 0
        return e

    def encode(self, tbs, rv, Qm, nbits, data):
        data = np.ascontiguousarray(data, np.uint8)
        e = np.zeros(nbits, np.uint8)
        assert self.lib.orc_dlsch_encode(tbs, rv, Qm, nbits, _ptr(data, _u8p), _ptr(e, _u8p)) == 0
        return e

    def softbuffer(self, max_cb):
        sb = OrcSoftbuffer()
        assert self.lib.orc_softbuffer_init(ctypes.byref(sb), max_cb) == 0
        return sb

    def reset(self, sb):
        self.lib.orc_softbuffer_reset(ctypes.byref(sb))

    def free(self, sb):
        self.lib.orc_softbuffer_free(ctypes.byref(sb))

    def decode(self, sb, tbs, rv, Qm, e, max_halfits):
        e = np.ascontiguousarray(e, np.int16)
        data = np.zeros(tbs // 8 + 8, np.uint8)
        noi = ctypes.c_uint32(0)
        r = self.lib.orc_dlsch_decode(ctypes.byref(sb), tbs, rv, Qm, e.size, _ptr(e, _i16p),
                                      _ptr(data, _u8p), max_halfits, ctypes.byref(noi))
        C = self.lib_segm_C(tbs)
        cb_crc = np.ctypeslib.as_array(sb.cb_crc, shape=(sb.max_cb,))[:C].copy()
        return r, data, noi.value, cb_crc

    def ulsch_decode(self, sb, tbs, rv, Qm, nof_symb, q_bits, max_halfits):
        """orc_ulsch_decode (srslte_ulsch_decode restated): -> (ret, data, noi, cb_crc)"""
        L = self.lib
        u32 = ctypes.c_uint32
        L.orc_ulsch_decode.argtypes = [ctypes.POINTER(OrcSoftbuffer), u32, u32, u32, u32, u32, _i16p,
                                       _u8p, u32, _u32p]
        q = np.ascontiguousarray(q_bits, np.int16)
        data = np.zeros(tbs // 8 + 8, np.uint8)
        noi = ctypes.c_uint32(0)
        r = L.orc_ulsch_decode(ctypes.byref(sb), tbs, rv, Qm, q.size, nof_symb, _ptr(q, _i16p),
                               _ptr(data, _u8p), max_halfits, ctypes.byref(noi))
        C = self.lib_segm_C(tbs)
        cb_crc = np.ctypeslib.as_array(sb.cb_crc, shape=(sb.max_cb,))[:C].copy()
        return r, data, noi.value, cb_crc

    def ulsch_deinterleave(self, q_bits, Qm, nof_symb):
        L = self.lib
        u32 = ctypes.c_uint32
        L.orc_ulsch_deinterleave.argtypes = [_i16p, u32, u32, u32, _i16p]
        q = np.ascontiguousarray(q_bits, np.int16)
        g = np.zeros(q.size, np.int16)
        assert L.orc_ulsch_deinterleave(_ptr(q, _i16p), Qm, q.size, nof_symb, _ptr(g, _i16p)) == 0
        return g

    def lib_segm_C(self, tbs):
        v = [ctypes.c_uint32(0) for _ in range(6)]
        self.lib.orc_cbsegm(tbs, *[ctypes.byref(x) for x in v])
        return v[0].value


class Ref(_Lib):
    def __init__(self):
        super().__init__(REF_SO, "ref_")
        L = self.lib
        L.ref_tdec_run_all_many.argtypes = [ctypes.c_int, _i16p, ctypes.c_size_t, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, _u8p]
        L.ref_cbsegm.argtypes = [ctypes.c_uint32, _u32p]

    def cbsegm(self, tbs):
        o = np.zeros(6, np.uint32)
        assert self.lib.ref_cbsegm(tbs, _ptr(o, _u32p)) == 0
        return tuple(int(x) for x in o)

    def tdec8_run(self, impl, sb_layout, inp, K, nhalf):
        L = self.lib
        L.ref_tdec8_run.argtypes = [ctypes.c_int, ctypes.c_int, _i8p, ctypes.c_size_t,
                                    ctypes.c_uint32, ctypes.c_uint32, _u8p]
        inp = np.ascontiguousarray(inp, dtype=np.int8)
        dec = np.zeros((nhalf, K // 8), np.uint8)
        assert L.ref_tdec8_run(impl, sb_layout, _ptr(inp, _i8p), inp.size, K, nhalf,
                               _ptr(dec, _u8p)) == 0
        return dec

    def tdec8_run16(self, impl, inp, K, nhalf):
        L = self.lib
        L.ref_tdec8_run16.argtypes = [ctypes.c_int, _i16p, ctypes.c_uint32, ctypes.c_uint32, _u8p]
        inp = np.ascontiguousarray(inp, dtype=np.int16)
        dec = np.zeros((nhalf, K // 8), np.uint8)
        assert L.ref_tdec8_run16(impl, _ptr(inp, _i16p), K, nhalf, _ptr(dec, _u8p)) == 0
        return dec

    # ---- DL-SCH (sch.c through ref_harness.c) ----
    def _dl_sigs(self):
        L = self.lib
        u32 = ctypes.c_uint32
        L.ref_rm_turbo_rx.argtypes = [_i16p, _i16p, u32, u32, u32, ctypes.c_int]
        L.ref_dlsch_encode.argtypes = [u32, u32, u32, u32, _u8p, _u8p, u32]
        L.ref_softbuffer_reset.argtypes = [ctypes.c_int, u32]
        L.ref_dlsch_decode.argtypes = [ctypes.c_int, u32, u32, u32, u32, _i16p, _u8p, u32, _u32p,
                                       _u8p]

    def rm_rx(self, e, out, K, rv, sb):
        self._dl_sigs()
        e = np.ascontiguousarray(e, np.int16)
        assert self.lib.ref_rm_turbo_rx(_ptr(e, _i16p), _ptr(out, _i16p), e.size, K, rv, sb) == 0
        return out

    def encode(self, tbs, rv, Qm, nbits, data, nof_prb=100):
        """-> unpacked e bits (the reference packs them, sch.c:281)"""
        self._dl_sigs()
        data = np.ascontiguousarray(data, np.uint8)
        e = np.zeros((nbits + 7) // 8 + 8, np.uint8)
        assert self.lib.ref_dlsch_encode(tbs, rv, Qm, nbits, _ptr(data, _u8p), _ptr(e, _u8p),
                                         nof_prb) == 0
        return np.unpackbits(e)[:nbits]

    def sb_reset(self, slot, nof_prb=100):
        self._dl_sigs()
        assert self.lib.ref_softbuffer_reset(slot, nof_prb) == 0

    def decode(self, slot, tbs, rv, Qm, e, max_halfits):
        self._dl_sigs()
        e = np.ascontiguousarray(e, np.int16)
        data = np.zeros(tbs // 8 + 8, np.uint8)
        noi = ctypes.c_uint32(0)
        crc = np.zeros(64, np.uint8)
        r = self.lib.ref_dlsch_decode(slot, tbs, rv, Qm, e.size, _ptr(e, _i16p), _ptr(data, _u8p),
                                      max_halfits, ctypes.byref(noi), _ptr(crc, _u8p))
        C = self.cbsegm(tbs)[0]
        return r, data, noi.value, crc[:C]


    # ---- UL-SCH (srslte_ulsch_encode / srslte_ulsch_decode through ref_harness.c) ----
    def ul_encode(self, tbs, rv, Qm, nbits, nof_symb, data, nof_prb=100):
        """-> unpacked q bits (after the channel interleaver)"""
        L = self.lib
        u32 = ctypes.c_uint32
        L.ref_ulsch_encode.argtypes = [u32, u32, u32, u32, u32, _u8p, _u8p, u32]
        data = np.ascontiguousarray(data, np.uint8)
        q = np.zeros((nbits + 7) // 8 + 8, np.uint8)
        assert L.ref_ulsch_encode(tbs, rv, Qm, nbits, nof_symb, _ptr(data, _u8p), _ptr(q, _u8p),
                                  nof_prb) == 0
        return np.unpackbits(q)[:nbits]

    def ul_decode(self, slot, tbs, rv, Qm, nof_symb, q_bits, max_halfits):
        L = self.lib
        u32 = ctypes.c_uint32
        L.ref_ulsch_decode.argtypes = [ctypes.c_int, u32, u32, u32, u32, u32, _i16p, _u8p, u32, _u32p,
                                       _u8p]
        q = np.ascontiguousarray(q_bits, np.int16)
        data = np.zeros(tbs // 8 + 8, np.uint8)
        noi = ctypes.c_uint32(0)
        crc = np.zeros(64, np.uint8)
        r = L.ref_ulsch_decode(slot, tbs, rv, Qm, q.size, nof_symb, _ptr(q, _i16p), _ptr(data, _u8p),
                               max_halfits, ctypes.byref(noi), _ptr(crc, _u8p))
        C = self.cbsegm(tbs)[0]
        return r, data, noi.value, crc[:C]

    # ---- UCI on the PUSCH (srslte_ulsch_uci_encode / the srslte_pusch_decode UCI steps) ----
    def uci_encode(self, u, data=None, nof_prb=100):
        """u: uci_case() dict -> unpacked q bits (UL-SCH with HARQ-ACK / RI / CQI multiplexed)"""
        L = self.lib
        u32 = ctypes.c_uint32
        L.ref_ulsch_uci_encode.argtypes = [u32] * 6 + [_u32p, _u32p, _u8p, u32, _u8p, _u8p, _u8p, u32]
        data = np.ascontiguousarray(data if data is not None else np.zeros(8, np.uint8), np.uint8)
        q = np.zeros((u["nof_bits"] + 7) // 8 + 8, np.uint8)
        I, O = np.array(u["I_off"], np.uint32), np.array(u["O"], np.uint32)
        ack, cqi = np.array(u["ack"], np.uint8), np.array(list(u["cqi"]) + [0], np.uint8)
        r = L.ref_ulsch_uci_encode(u["tbs"], u["Qm"], u["nof_bits"], u["nof_symb"], u["M_sc"], u["M_sc_init"],
                                   _ptr(I, _u32p), _ptr(O, _u32p), _ptr(ack, _u8p), u["ri"], _ptr(cqi, _u8p),
                                   _ptr(data, _u8p), _ptr(q, _u8p), nof_prb)
        assert r == 0, r
        return np.unpackbits(q)[:u["nof_bits"]]

    def uci_decode(self, slot, u, q_scrambled, c, max_halfits=8):
        """the reference's UCI + data decode of scrambled soft bits -> (ret, out[4 + O_cqi], g, data, noi, cb_crc)"""
        L = self.lib
        u32 = ctypes.c_uint32
        L.ref_ulsch_uci_decode.argtypes = ([ctypes.c_int] + [u32] * 7 + [_u32p, _u32p, _i16p, _u8p, _u8p, u32, _u32p,
                                           _u8p, _u8p, _i16p])
        q = np.ascontiguousarray(q_scrambled, np.int16)
        c = np.ascontiguousarray(c, np.uint8)
        I, O = np.array(u["I_off"], np.uint32), np.array(u["O"], np.uint32)
        data = np.zeros(u["tbs"] // 8 + 8, np.uint8)
        out = np.zeros(4 + u["O"][2] + 4, np.uint8)
        g = np.zeros(u["nof_bits"] + 8, np.int16)
        noi = ctypes.c_uint32(0)
        crc = np.zeros(64, np.uint8)
        r = L.ref_ulsch_uci_decode(slot, u["tbs"], u["rv"], u["Qm"], u["nof_bits"], u["nof_symb"], u["M_sc"],
                                   u["M_sc_init"], _ptr(I, _u32p), _ptr(O, _u32p), _ptr(q, _i16p), _ptr(c, _u8p),
                                   _ptr(data, _u8p), max_halfits, ctypes.byref(noi), _ptr(crc, _u8p),
                                   _ptr(out, _u8p), _ptr(g, _i16p))
        C = self.cbsegm(u["tbs"])[0] if u["tbs"] else 0
        return r, out[:4 + u["O"][2]], g[:u["nof_bits"]], data, noi.value, crc[:C]


def uci_case(tbs, Qm, nof_prb_alloc, nof_symb=12, O=(1, 1, 0), I_off=(0, 2, 2), ack=(1, 0), ri=1, cqi=(), rv=0,
             M_sc_init=None):
    """a PUSCH configuration with UCI: M_sc = 12 nof_prb_alloc, H' = M_sc N_symb, nof_bits = H' Qm"""
    M_sc = 12 * nof_prb_alloc
    return dict(tbs=tbs, rv=rv, Qm=Qm, nof_symb=nof_symb, M_sc=M_sc, M_sc_init=M_sc_init or M_sc,
                nof_bits=M_sc * nof_symb * Qm, O=tuple(O), I_off=tuple(I_off), ack=tuple(ack), ri=ri, cqi=tuple(cqi))


def orc_ulsch_uci(oracle, u, q_scrambled, c):
    """the oracle's UCI steps -> (ret, out[4 + O_cqi], g, (Q'_ack, Q'_ri, Q'_cqi))"""
    L = oracle.lib
    u32 = ctypes.c_uint32
    L.orc_ulsch_uci.argtypes = [u32] * 6 + [_u32p, _u32p, _i16p, _u8p, _u8p, _i16p, _u32p]
    q = np.ascontiguousarray(q_scrambled, np.int16)
    c = np.ascontiguousarray(c, np.uint8)
    I, O = np.array(u["I_off"], np.uint32), np.array(u["O"], np.uint32)
    out = np.zeros(4 + u["O"][2] + 4, np.uint8)
    g = np.zeros(u["nof_bits"] + 8, np.int16)
    qp = np.zeros(3, np.uint32)
    r = L.orc_ulsch_uci(u["tbs"], u["Qm"], u["nof_bits"], u["nof_symb"], u["M_sc"], u["M_sc_init"], _ptr(I, _u32p),
                        _ptr(O, _u32p), _ptr(q, _i16p), _ptr(c, _u8p), _ptr(out, _u8p), _ptr(g, _i16p), _ptr(qp, _u32p))
    return r, out[:4 + u["O"][2]], g[:u["nof_bits"]], tuple(int(v) for v in qp)


def uci_rx(rng, q_bits, c, amp=40, sigma=25):
    """received soft bits of transmitted q bits: LLR = (2b - 1) amp + noise (int16; srsLTE's soft
    demapper gives bit 0 a negative value), then scrambled by c (negated where c = 1), as the PUSCH
    receiver holds them before descrambling"""
    llr = (2 * q_bits.astype(np.int32) - 1) * amp + np.round(rng.normal(0, sigma, q_bits.size)).astype(np.int32)
    llr = np.clip(llr, -32768, 32767).astype(np.int16)
    return np.where(c.astype(bool), -llr, llr).astype(np.int16)


def have_ref():
    return os.path.exists(REF_SO)


REF_FRONT = os.path.join(REPO, "oracle", "_ref", "ref_front")


def have_ref_front():
    return os.path.exists(REF_FRONT)


def _run_ref_front(mode, payload):
    """run oracle/_ref/ref_front (the reference's chest_dl.c / ue_dl.c, this container only) on one
    request; -> the response bytes"""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fi, fo = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fi, "wb") as f:
            f.write(payload)
        r = subprocess.run([REF_FRONT, mode, fi, fo], capture_output=True, text=True)
        assert r.returncode == 0, "ref_front %s failed (%d): %s" % (mode, r.returncode, r.stderr[-2000:])
        with open(fo, "rb") as f:
            return f.read()


def ref_front_chest(nof_prb, cell_id, nports, nrx, sfs, grids, filt=(0.1, 0.8, 0.1), gauss=None,
                    smooth_auto=False, average=False, noise_alg=0, rsrp_neighbour=True, cfo_enable=True,
                    cfo_mask=0x3FF, noise_init=0.0, cp=0):
    """srslte_chest_dl_* of the reference on ONE estimator over the subframe sequence sfs; grids[i][a]
    complex64 [14 * 12 nof_prb] (12 * 12 nof_prb for an extended-CP cell, cp=1). filt: explicit filter (srslte_chest_dl_set_smooth_filter), or
    gauss=(order, std) for srslte_chest_dl_set_smooth_filter_gauss. -> list per subframe of dict(
    noise_before [nrx][np], ce [nrx][np][n], noise / rsrp / rssi / rsrp_corr / cfo [nrx][np],
    getters [noise, snr, rssi, rsrq, rsrp, rsrp_neighbour, cfo])"""
    n = (12 if cp else 14) * 12 * nof_prb
    f = np.zeros(32, np.float32)
    f[:len(filt)] = filt
    head = np.array([nof_prb, cell_id, nports | (cp << 8), nrx, len(sfs), 1 if gauss else 0, len(filt)],
                    np.uint32).tobytes()
    head += f.tobytes()
    head += np.array([gauss[0] if gauss else 0], np.uint32).tobytes()
    head += np.array([gauss[1] if gauss else 0.0], np.float32).tobytes()
    head += np.array([int(smooth_auto), int(average), noise_alg, int(rsrp_neighbour), int(cfo_enable), cfo_mask],
                     np.uint32).tobytes()
    head += np.array([noise_init], np.float32).tobytes()
    body = b"".join(np.array([sf], np.uint32).tobytes() +
                    b"".join(np.ascontiguousarray(grids[i][a], np.complex64).tobytes() for a in range(nrx))
                    for i, sf in enumerate(sfs))
    raw = _run_ref_front("chest", head + body)
    out, o, m = [], 0, nrx * nports
    for _ in sfs:
        nb = np.frombuffer(raw, np.float32, m, o).reshape(nrx, nports).copy()
        o += 4 * m
        ce = np.frombuffer(raw, np.complex64, m * n, o).reshape(nrx, nports, n).copy()
        o += 8 * m * n
        meas = np.frombuffer(raw, np.float32, 5 * m, o).reshape(nrx, nports, 5).copy()
        o += 20 * m
        get = np.frombuffer(raw, np.float32, 7, o).copy()
        o += 28
        out.append(dict(noise_before=nb, ce=ce, noise=meas[..., 0], rsrp=meas[..., 1], rssi=meas[..., 2],
                        rsrp_corr=meas[..., 3], cfo=meas[..., 4], getters=get))
    assert o == len(raw)
    return out


def ref_front_dci(nof_prb, cell_id, nports, nrx, phich_len, phich_res, subframes):
    """srslte_pdcch_extract_llr_multi + srslte_ue_dl_find_dl_dci(_type) + srslte_ue_dl_find_ul_dci +
    srslte_dci_msg_to_ul_grant of the reference (ue_dl.c on ONE srslte_ue_dl_t, in phch_worker's order)
    over a subframe sequence. subframes: dicts with sf_idx, cfi, noise, rnti, tm, rnti_type, ul_rnti
    (0: no UL search), n_rb_ho, y [nrx] and h [nports][nrx] (complex64, zero-padded to 14 * 12 nof_prb).
    -> per subframe dict(llr, dl=(found, format, L, ncce, nof_bits, buf), ul=(...), ul_grant=(ret,
    dci 11 fields, grant 10 fields), pending)"""
    n = 14 * 12 * nof_prb
    pad = lambda a: np.concatenate([np.asarray(a, np.complex64), np.zeros(n - len(a), np.complex64)])
    pay = np.array([nof_prb, cell_id, nports, nrx, phich_len, phich_res, len(subframes)], np.uint32).tobytes()
    for s in subframes:
        pay += np.array([s["sf_idx"], s["cfi"]], np.uint32).tobytes()
        pay += np.array([s["noise"]], np.float32).tobytes()
        pay += np.array([s["rnti"], s["tm"], s["rnti_type"], s.get("ul_rnti", 0), s.get("n_rb_ho", 0)],
                        np.int64).astype(np.uint32).tobytes()
        pay += b"".join(pad(s["y"][a]).tobytes() for a in range(nrx))
        pay += b"".join(pad(s["h"][p][a]).tobytes() for p in range(nports) for a in range(nrx))
    raw = _run_ref_front("dci", pay)
    out, o = [], 0

    def msg():
        nonlocal o
        v = np.frombuffer(raw, np.int32, 5, o)
        o += 20
        buf = np.frombuffer(raw, np.uint8, 128, o).copy()
        o += 128
        return (int(v[0]), int(v[1]), int(v[2]), int(v[3]), int(v[4]), buf if v[0] > 0 else buf[:0])

    for _ in subframes:
        nl = int(np.frombuffer(raw, np.int32, 1, o)[0])
        o += 4
        llr = np.frombuffer(raw, np.float32, nl, o).copy()
        o += 4 * nl
        dl, ul = msg(), msg()
        g = np.frombuffer(raw, np.int32, 23, o).copy()
        o += 92
        out.append(dict(llr=llr, dl=dl, ul=ul, ul_grant=(int(g[0]), g[1:12], g[12:22]), pending=int(g[22])))
    assert o == len(raw)
    return out


def ref_front_ue_dl(nof_prb, cell_id, nports, nrx, phich_len, phich_res, max_prb, rnti, tm, ttis, grids,
                    filt=None, gauss=None, average=False, noise_alg=0, rsrp_neighbour=False, cfo_enable=False,
                    cfo_mask=0):
    """srslte_ue_dl_decode_rnti's steps after the FFT (ue_dl.c:467-620: chest, PCFICH, PDCCH, DL DCI search,
    grant, PDSCH) of the reference on ONE ue_dl-shaped object over a subframe sequence, then the
    estimator getters and the TM3 / TM4 feedback phch_worker reads; grids[i][a] complex64
    [14 * 12 nof_prb]. Estimator settings as ref_front_chest (filt / gauss None: srslte_chest_dl_init's
    default filter). -> per subframe dict(cfi, corr, noise, dl=(found, format, L, ncce, nof_bits, buf),
    ret, tbs, rv, mod, ack, noi, nre, data [12000] u8, ce [nports][nrx][n], getters [noise, snr, rssi,
    rsrq, rsrp, rsrp_neighbour, cfo], cn, ri_tm3, ret_cn, ri, pmi, pmi_l [2], ret_pmi, sinr [2][4])"""
    n = 14 * 12 * nof_prb
    pay = np.array([nof_prb, cell_id, nports, nrx, phich_len, phich_res, max_prb, rnti, tm, len(ttis)],
                   np.uint32).tobytes()
    f = np.zeros(32, np.float32)
    if filt is not None:
        f[:len(filt)] = filt
    mode = 1 if gauss else 0 if filt is not None else 2
    pay += np.array([mode, len(filt) if filt is not None else 0], np.uint32).tobytes() + f.tobytes()
    pay += np.array([gauss[0] if gauss else 0], np.uint32).tobytes()
    pay += np.array([gauss[1] if gauss else 0.0], np.float32).tobytes()
    pay += np.array([int(average), noise_alg, int(rsrp_neighbour), int(cfo_enable), cfo_mask], np.uint32).tobytes()
    for i, t in enumerate(ttis):
        pay += np.array([t], np.uint32).tobytes()
        pay += b"".join(np.ascontiguousarray(grids[i][a], np.complex64).tobytes() for a in range(nrx))
    raw = _run_ref_front("ue_dl", pay)
    out, o = [], 0
    for _ in ttis:
        cfi = int(np.frombuffer(raw, np.int32, 1, o)[0])
        corr, noise = np.frombuffer(raw, np.float32, 2, o + 4)
        o += 12
        v = np.frombuffer(raw, np.int32, 5, o)
        o += 20
        buf = np.frombuffer(raw, np.uint8, 128, o).copy()
        o += 128
        r = np.frombuffer(raw, np.int32, 7, o)
        o += 28
        data = np.frombuffer(raw, np.uint8, 12000, o).copy()
        o += 12000
        ce = np.frombuffer(raw, np.complex64, nports * nrx * n, o).reshape(nports, nrx, n).copy()
        o += 8 * nports * nrx * n
        get = np.frombuffer(raw, np.float32, 7, o).copy()
        o += 28
        cn = float(np.frombuffer(raw, np.float32, 1, o)[0])
        fb = np.frombuffer(raw, np.int32, 7, o + 4)
        o += 32
        sinr = np.frombuffer(raw, np.float32, 8, o).reshape(2, 4).copy()
        o += 32
        out.append(dict(cfi=cfi, corr=float(corr), noise=float(noise),
                        dl=(int(v[0]), int(v[1]), int(v[2]), int(v[3]), int(v[4]), buf if v[0] > 0 else buf[:0]),
                        ret=int(r[0]), tbs=int(r[1]), rv=int(r[2]), mod=int(r[3]), ack=int(r[4]), noi=int(r[5]),
                        nre=int(r[6]), data=data, ce=ce, getters=get, cn=cn, ri_tm3=int(fb[0]), ret_cn=int(fb[1]),
                        ri=int(fb[2]), pmi=int(fb[3]), pmi_l=[int(fb[4]), int(fb[5])], ret_pmi=int(fb[6]),
                        sinr=sinr))
    assert o == len(raw)
    return out


# ------------------------------------------------------------------ synthetic data ----

def cb_sizes():
    from itertools import chain
    return list(chain(range(40, 512, 8), range(512, 1024, 16), range(1024, 2048, 32),
                      range(2048, 6145, 64)))


def awgn_llr(coded_bits, ebno_db, rng, scale=100.0):
    """BPSK over AWGN and int16 LLR quantisation as turbodecoder_test.c:236-252:
    llr = (int16)(100*(+-1 + sigma*n)), sigma from Eb/N0 at rate 1/3 (ch_awgn.c:36-39)."""
    esno_db = ebno_db + 10.0 * np.log10(1.0 / 3.0)
    sigma = np.float32(np.sqrt(1.0 / (10.0 ** (esno_db / 10.0))))
    sym = np.where(coded_bits.astype(bool), np.float32(1.0), np.float32(-1.0))
    y = sym + sigma * rng.standard_normal(coded_bits.size).astype(np.float32)
    return (np.float32(scale) * y).astype(np.int16)


def awgn_llr8(coded_bits, ebno_db, rng, scale=20.0):
    """as awgn_llr, quantised to int8 with saturation (the 8-bit LLR path)"""
    esno_db = ebno_db + 10.0 * np.log10(1.0 / 3.0)
    sigma = np.float32(np.sqrt(1.0 / (10.0 ** (esno_db / 10.0))))
    sym = np.where(coded_bits.astype(bool), np.float32(1.0), np.float32(-1.0))
    y = sym + sigma * rng.standard_normal(coded_bits.size).astype(np.float32)
    return np.clip(np.rint(np.float32(scale) * y), -128, 127).astype(np.int8)


def make_cb8(K, ebno_db, seed, scale=20.0, oracle=None):
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2, K, dtype=np.uint8)
    coded = (oracle or Oracle()).tcod_encode(bits)
    return bits, awgn_llr8(coded, ebno_db, rng, scale)


def natural_to_sb(inp_nat, K, nsb):
    """[s,p0,p1]*K + 12 tail (natural) -> rm_turbo's sub-block layout: stream s at s*(K+32),
    SB index k*nsb+d = natural position d*(K/nsb)+k, tail at 3*(K+32) (rm_turbo.c:239-264)."""
    L = K // nsb
    out = np.zeros(3 * (K + 32) + 12, inp_nat.dtype)
    p = np.arange(K)
    sbidx = (p % L) * nsb + p // L
    for s in range(3):
        out[s * (K + 32) + sbidx] = inp_nat[3 * p + s]
    out[3 * (K + 32):] = inp_nat[3 * K:3 * K + 12]
    return out


def make_cb(K, ebno_db, seed, oracle=None):
    """Random bits -> turbo encode (oracle restatement of turbocoder.c) -> AWGN -> int16 LLR."""
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2, K, dtype=np.uint8)
    o = oracle or Oracle()
    coded = o.tcod_encode(bits)
    return bits, awgn_llr(coded, ebno_db, rng)


def pack_bits(bits):
    """bits (0/1, MSB first) -> bytes, as srslte_bit_pack_vector."""
    return np.packbits(np.asarray(bits, np.uint8))


def make_crc_cb(K, ebno_db, seed, poly=CRC24B, oracle=None):
    """Code block whose last 24 bits are the CRC of the first K-24 (TS 36.212 5.1.1/5.1.2),
    so the CRC over all K decoded bits is 0 exactly when decoding succeeds."""
    o = oracle or Oracle()
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 2, K - 24, dtype=np.uint8)
    crc = o.crc(poly, pack_bits(data), K - 24)
    crcbits = np.array([(crc >> (23 - i)) & 1 for i in range(24)], np.uint8)
    bits = np.concatenate([data, crcbits])
    coded = o.tcod_encode(bits)
    return bits, awgn_llr(coded, ebno_db, rng)


# ------------------------------------------------------------------ PDSCH front-end ----
_f32p = ctypes.POINTER(ctypes.c_float)
MOD_BPSK, MOD_QPSK, MOD_16QAM, MOD_64QAM = 0, 1, 2, 3
BITS_PER_SYMBOL = {MOD_BPSK: 1, MOD_QPSK: 2, MOD_16QAM: 4, MOD_64QAM: 6}


class PdschOracle:
    """Bindings of oracle/pdsch_oracle.c (RE map, SISO equaliser, soft demapper, scrambling)."""

    def __init__(self, oracle):
        L = self.lib = oracle.lib
        u32 = ctypes.c_uint32
        L.orc_pdsch_re_map.argtypes = [u32, u32, u32, u32, u32, _u8p, _u32p]
        L.orc_predecode_single.argtypes = [_f32p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_float,
                                           ctypes.c_float]
        L.orc_demod_s.argtypes = [ctypes.c_int, _f32p, ctypes.c_int, _i16p]
        L.orc_sequence.argtypes = [u32, u32, _u8p]
        L.orc_pdsch_seed.argtypes = [ctypes.c_uint16, ctypes.c_int, u32, u32]
        L.orc_pdsch_seed.restype = u32
        L.orc_scramble_s.argtypes = [u32, _i16p, u32]
        L.orc_csi_correction.argtypes = [ctypes.c_int, _f32p, ctypes.c_int, _i16p]
        L.orc_predecode_ccd_2x2.argtypes = [_f32p] * 10 + [ctypes.c_int, ctypes.c_float, ctypes.c_float]

    def predecode_ccd(self, y, h, scaling=1.0, noise=0.0, csi=False):
        """TM3 CDD 2x2 MMSE: y [2 rx][n], h [2 ports][2 rx][n] -> x [2 layers][n] (+ csi [2][n])"""
        y = [np.ascontiguousarray(v, np.complex64) for v in y]
        hh = [np.ascontiguousarray(h[p][a], np.complex64) for p in (0, 1) for a in (0, 1)]
        n = y[0].size
        x = [np.zeros(n, np.complex64) for _ in range(2)]
        c = [np.zeros(n, np.float32) for _ in range(2)] if csi else [None, None]
        self.lib.orc_predecode_ccd_2x2(*[v.ctypes.data_as(_f32p) for v in y + hh + x],
                                       _ptr(c[0], _f32p), _ptr(c[1], _f32p), n, scaling, noise)
        return (x, c) if csi else x

    def predecode_multiplex(self, y, h, codebook, layers, scaling=1.0, noise=0.0, csi=False, lib=None):
        """TM4 spatial multiplexing (orc_predecode_multiplex, or ref_predecode_multiplex when lib is
        the reference build): y [2 rx][n], h [2 ports][2 rx][n] -> x [layers][n] (+ csi)"""
        L = lib.lib if lib is not None else self.lib
        name = "ref_predecode_multiplex" if lib is not None else "orc_predecode_multiplex"
        f = getattr(L, name)
        f.argtypes = [_f32p] * 10 + [ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int]
        y = [np.ascontiguousarray(v, np.complex64) for v in y]
        hh = [np.ascontiguousarray(h[p][a], np.complex64) for p in (0, 1) for a in (0, 1)]
        n = y[0].size
        x = [np.zeros(n, np.complex64) for _ in range(2)]
        c = [np.zeros(n, np.float32) for _ in range(2)] if csi else [None, None]
        r = f(*[v.ctypes.data_as(_f32p) for v in y + hh + x], _ptr(c[0], _f32p), _ptr(c[1], _f32p), n, scaling,
              noise, codebook, layers)
        assert r == 0, r
        x, c = x[:layers], c[:layers]
        return (x, c) if csi else x

    def csi_correction(self, mod, csi, llr):
        csi = np.ascontiguousarray(csi, np.float32)
        llr = np.array(llr, np.int16)
        assert self.lib.orc_csi_correction(mod, csi.ctypes.data_as(_f32p), csi.size, _ptr(llr, _i16p)) == 0
        return llr

    def re_map(self, nof_prb, cell_id, nof_ports, lstart, sf_idx, prb_mask):
        m = np.ascontiguousarray(prb_mask, np.uint8).reshape(-1)
        idx = np.zeros(nof_prb * 12 * 14, np.uint32)
        n = self.lib.orc_pdsch_re_map(nof_prb, cell_id, nof_ports, lstart, sf_idx, _ptr(m, _u8p),
                                      _ptr(idx, _u32p))
        return idx[:n]

    def predecode(self, y, h, scaling=1.0, noise=0.0, csi=False):
        y = np.ascontiguousarray(y, np.complex64)
        h = np.ascontiguousarray(h, np.complex64)
        x = np.zeros_like(y)
        c = np.zeros(y.size, np.float32) if csi else None
        self.lib.orc_predecode_single(y.ctypes.data_as(_f32p), h.ctypes.data_as(_f32p),
                                      x.ctypes.data_as(_f32p), _ptr(c, _f32p), y.size, scaling, noise)
        return (x, c) if csi else x

    def demod(self, mod, sym):
        sym = np.ascontiguousarray(sym, np.complex64)
        llr = np.zeros(sym.size * BITS_PER_SYMBOL[mod], np.int16)
        assert self.lib.orc_demod_s(mod, sym.ctypes.data_as(_f32p), sym.size, _ptr(llr, _i16p)) == 0
        return llr

    def seed(self, rnti, q, nslot, cell_id):
        return self.lib.orc_pdsch_seed(rnti, q, nslot, cell_id)

    def sequence(self, seed, n):
        c = np.zeros(n, np.uint8)
        assert self.lib.orc_sequence(seed, n, _ptr(c, _u8p)) == 0
        return c

    def scramble(self, seed, llr):
        llr = np.array(llr, np.int16)
        assert self.lib.orc_scramble_s(seed, _ptr(llr, _i16p), llr.size) == 0
        return llr


def ref_pdsch(ref):
    """Attach the PDSCH front-end harness signatures to a Ref instance."""
    L = ref.lib
    u32 = ctypes.c_uint32
    L.ref_demod_s.argtypes = [ctypes.c_int, _f32p, ctypes.c_int, _i16p]
    L.ref_sequence_pdsch.argtypes = [ctypes.c_uint16, ctypes.c_int, u32, u32, u32, _u8p]
    L.ref_scramble_pdsch_s.argtypes = [ctypes.c_uint16, ctypes.c_int, u32, u32, _i16p, u32]
    L.ref_predecode_single.argtypes = [_f32p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_float,
                                       ctypes.c_float]
    L.ref_pdsch_get.argtypes = [u32, u32, u32, u32, u32, _u8p, _f32p, _f32p]
    L.ref_predecode_ccd.argtypes = [_f32p] * 10 + [ctypes.c_int, ctypes.c_float, ctypes.c_float]
    return L


def ref_predecode_ccd(L, y, h, scaling=1.0, noise=0.0, csi=False):
    """the reference's srslte_predecoding_ccd_mmse (AVX2 body + C tail) on the same arguments"""
    y = [np.ascontiguousarray(v, np.complex64) for v in y]
    hh = [np.ascontiguousarray(h[p][a], np.complex64) for p in (0, 1) for a in (0, 1)]
    n = y[0].size
    x = [np.zeros(n, np.complex64) for _ in range(2)]
    c = [np.zeros(n, np.float32) for _ in range(2)] if csi else [None, None]
    assert L.ref_predecode_ccd(*[v.ctypes.data_as(_f32p) for v in y + hh + x],
                               _ptr(c[0], _f32p), _ptr(c[1], _f32p), n, scaling, noise) == 0
    return (x, c) if csi else x


# ------------------------------------------------------------------ 8-bit LLR chain ----
class Llr8:
    """The llr_is_8bit receive chain (pdsch.c:795-806, sch.c:344-364): int8 soft demapping,
    int8 scrambling, the 8-bit CSI weighting, 8-bit de-rate-matching and the DL-SCH decode on int8
    softbuffer rows. `lib` is the oracle (prefix orc_) or the reference harness (prefix ref_)."""

    def __init__(self, lib, ref=False):
        L = self.lib = lib.lib if hasattr(lib, "lib") else lib
        self.ref = ref
        u32 = ctypes.c_uint32
        if ref:
            L.ref_demod_b.argtypes = [ctypes.c_int, _f32p, ctypes.c_int, _i8p]
            L.ref_scramble_pdsch_sb.argtypes = [ctypes.c_uint16, ctypes.c_int, u32, u32, _i8p, u32]
            L.ref_rm_turbo_rx_8bit.argtypes = [_i8p, _i8p, u32, u32, u32]
            L.ref_dlsch_decode8.argtypes = [ctypes.c_int, u32, u32, u32, u32, _i8p, _u8p, u32, _u32p,
                                            _u8p]
            L.ref_softbuffer_reset.argtypes = [ctypes.c_int, u32]
            L.ref_cbsegm.argtypes = [u32, _u32p]
        else:
            L.orc_demod_b.argtypes = [ctypes.c_int, _f32p, ctypes.c_int, _i8p]
            L.orc_scramble_sb.argtypes = [u32, _i8p, u32]
            L.orc_pdsch_seed.argtypes = [ctypes.c_uint16, ctypes.c_int, u32, u32]
            L.orc_pdsch_seed.restype = u32
            L.orc_csi_correction_b.argtypes = [ctypes.c_int, _f32p, ctypes.c_int, _i8p]
            L.orc_rm_turbo_rx_8bit.argtypes = [_i8p, _i8p, u32, u32, u32]
            L.orc_dlsch_decode8.argtypes = [ctypes.POINTER(OrcSoftbuffer), u32, u32, u32, u32, _i8p,
                                            _u8p, u32, _u32p]
            L.orc_cbsegm.argtypes = [u32] + [_u32p] * 6

    def demod(self, mod, sym):
        sym = np.ascontiguousarray(sym, np.complex64)
        llr = np.zeros(sym.size * BITS_PER_SYMBOL[mod], np.int8)
        f = self.lib.ref_demod_b if self.ref else self.lib.orc_demod_b
        assert f(mod, sym.ctypes.data_as(_f32p), sym.size, _ptr(llr, _i8p)) == 0
        return llr

    def scramble(self, rnti, q, nslot, cell_id, llr):
        llr = np.array(llr, np.int8)
        if self.ref:
            assert self.lib.ref_scramble_pdsch_sb(rnti, q, nslot, cell_id, _ptr(llr, _i8p), llr.size) == 0
        else:
            seed = self.lib.orc_pdsch_seed(rnti, q, nslot, cell_id)
            assert self.lib.orc_scramble_sb(seed, _ptr(llr, _i8p), llr.size) == 0
        return llr

    def csi_correction(self, mod, csi, llr):
        csi = np.ascontiguousarray(csi, np.float32)
        llr = np.array(llr, np.int8)
        assert self.lib.orc_csi_correction_b(mod, csi.ctypes.data_as(_f32p), csi.size, _ptr(llr, _i8p)) == 0
        return llr

    def rm_rx(self, e, out, K, rv):
        e = np.ascontiguousarray(e, np.int8)
        f = self.lib.ref_rm_turbo_rx_8bit if self.ref else self.lib.orc_rm_turbo_rx_8bit
        assert f(_ptr(e, _i8p), _ptr(out, _i8p), e.size, K, rv) == 0
        return out

    def segm_C(self, tbs):
        o = np.zeros(6, np.uint32)
        if self.ref:
            self.lib.ref_cbsegm(tbs, _ptr(o, _u32p))
            return int(o[0])
        v = [ctypes.c_uint32(0) for _ in range(6)]
        self.lib.orc_cbsegm(tbs, *[ctypes.byref(x) for x in v])
        return v[0].value

    def decode(self, sb, tbs, rv, Qm, e, max_halfits):
        """sb: an OrcSoftbuffer (oracle) or a reference HARQ slot number"""
        e = np.ascontiguousarray(e, np.int8)
        data = np.zeros(tbs // 8 + 8, np.uint8)
        noi = ctypes.c_uint32(0)
        C = self.segm_C(tbs)
        if self.ref:
            crc = np.zeros(64, np.uint8)
            r = self.lib.ref_dlsch_decode8(sb, tbs, rv, Qm, e.size, _ptr(e, _i8p), _ptr(data, _u8p),
                                           max_halfits, ctypes.byref(noi), _ptr(crc, _u8p))
            return r, data, noi.value, crc[:C]
        r = self.lib.orc_dlsch_decode8(ctypes.byref(sb), tbs, rv, Qm, e.size, _ptr(e, _i8p),
                                       _ptr(data, _u8p), max_halfits, ctypes.byref(noi))
        cb_crc = np.ctypeslib.as_array(sb.cb_crc, shape=(sb.max_cb,))[:C].copy()
        return r, data, noi.value, cb_crc


# ------------------------------------------------------------------ TM2 transmit diversity ----
def predecode_txdiv(lib, y, h, scaling=1.0, csi=False, ref=False):
    """srslte_predecoding_diversity_multi (2 or 4 ports) + srslte_layerdemap_diversity: y [nrx][n],
    h [ports][nrx][n] -> d [n] (+ csi [n]); lib: the oracle (orc_) or the reference (ref_)"""
    L = lib.lib if hasattr(lib, "lib") else lib
    if len(h) == 4:
        f = getattr(L, "ref_predecode_txdiv4" if ref else "orc_predecode_txdiv4")
        f.argtypes = [ctypes.POINTER(_f32p), ctypes.POINTER(_f32p), ctypes.c_int, ctypes.c_int, ctypes.c_float,
                      _f32p, _f32p]
        nrx = len(y)
        ys = [np.ascontiguousarray(v, np.complex64) for v in y]
        hs = [np.ascontiguousarray(h[p][a], np.complex64) if a < nrx else None for p in range(4) for a in (0, 1)]
        n = ys[0].size
        d = np.zeros(n, np.complex64)
        c = np.zeros(n, np.float32) if csi else None
        P = lambda a: a.ctypes.data_as(_f32p) if a is not None else None
        ya = (_f32p * 2)(*[P(v) for v in ys + [None] * (2 - nrx)])
        ha = (_f32p * 8)(*[P(v) for v in hs])
        assert f(ya, ha, nrx, n, scaling, P(d), P(c)) == 0
        return (d, c) if csi else d
    f = getattr(L, "ref_predecode_txdiv" if ref else "orc_predecode_txdiv")
    f.argtypes = [_f32p] * 6 + [ctypes.c_int, ctypes.c_int, ctypes.c_float, _f32p, _f32p]
    nrx = len(y)
    ys = [np.ascontiguousarray(v, np.complex64) for v in y] + [None] * (2 - nrx)
    hs = [np.ascontiguousarray(h[p][a], np.complex64) if a < nrx else None for p in (0, 1) for a in (0, 1)]
    n = ys[0].size
    d = np.zeros(n, np.complex64)
    c = np.zeros(n, np.float32) if csi else None
    P = lambda a: a.ctypes.data_as(_f32p) if a is not None else None
    assert f(P(ys[0]), P(ys[1]), *[P(v) for v in hs], nrx, n, scaling, P(d), P(c)) == 0
    return (d, c) if csi else d


# ------------------------------------------------------------------ PDCCH Viterbi ----
def viterbi_tb_decode_f(lib, sym, F, ref=False):
    """srslte_viterbi_decode_f (tail-biting K=7 r=1/3, PDCCH polynomials): 3F floats -> F bits"""
    L = lib.lib if hasattr(lib, "lib") else lib
    f = getattr(L, "ref_viterbi37_tb_decode_f" if ref else "orc_viterbi37_tb_decode_f")
    f.argtypes = [_f32p, ctypes.c_uint32, _u8p]
    sym = np.ascontiguousarray(sym, np.float32)
    out = np.zeros(F, np.uint8)
    assert f(sym.ctypes.data_as(_f32p), F, _ptr(out, _u8p)) == 0
    return out


def dci_decode(lib, e, nof_bits, ref=False):
    """srslte_pdcch_decode_msg's decode of one candidate: (decoded 0/1, bits[nof_bits+16], crc_rem)"""
    L = lib.lib if hasattr(lib, "lib") else lib
    f = getattr(L, "ref_dci_decode" if ref else "orc_dci_decode")
    f.argtypes = [_f32p, ctypes.c_uint32, ctypes.c_uint32, _u8p, ctypes.POINTER(ctypes.c_uint16)]
    e = np.ascontiguousarray(e, np.float32)
    d = np.zeros(nof_bits + 16, np.uint8)
    c = ctypes.c_uint16(0)
    r = f(e.ctypes.data_as(_f32p), e.size, nof_bits, _ptr(d, _u8p), ctypes.byref(c))
    assert r in (0, 1)
    return r, d, c.value


# ------------------------------------------------------------------ PCFICH ----
def pcfich_re_map(lib, nof_prb, cell_id, ref=False):
    """the 16 RE indices of symbol 0 (srslte_regs_pcfich_get order)"""
    L = lib.lib if hasattr(lib, "lib") else lib
    idx = np.zeros(16, np.uint32)
    if ref:
        f = L.ref_pcfich
        f.argtypes = [ctypes.c_uint32] * 4 + [_f32p] * 6 + [ctypes.c_float, ctypes.c_uint32, _u32p,
                                                            _f32p, _u32p]
        assert f(nof_prb, cell_id, 1, 1, None, None, None, None, None, None, 0.0, 0, None, None,
                 _ptr(idx, _u32p)) == 16
    else:
        f = L.orc_pcfich_re_map
        f.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _u32p]
        assert f(nof_prb, cell_id, _ptr(idx, _u32p)) == 16
    return idx


def pcfich_decode(lib, nof_prb, cell_id, nports, nrx, y, h, noise, sf_idx, ref=False):
    """srslte_pcfich_decode_multi: y[a] complex64 subframe grids, h[p][a] estimates -> (cfi, corr)"""
    L = lib.lib if hasattr(lib, "lib") else lib
    n = nof_prb * 12 * 14
    pad = lambda a: np.ascontiguousarray(np.concatenate([a, np.zeros(n - a.size, np.complex64)])
                                         if a.size < n else a, np.complex64)
    ys = [pad(y[a]) for a in range(nrx)]
    hs = [[pad(h[p][a]) for a in range(nrx)] for p in range(nports)]
    P = lambda a: a.ctypes.data_as(_f32p) if a is not None else None
    cfi, corr = ctypes.c_uint32(0), ctypes.c_float(0)
    if ref and nports == 4:
        f = L.ref_pcfich_n
        f.argtypes = [ctypes.c_uint32] * 4 + [ctypes.POINTER(_f32p), ctypes.POINTER(_f32p), ctypes.c_float,
                                              ctypes.c_uint32, _u32p, _f32p]
        ya = (_f32p * 2)(*[P(v) for v in ys] + [None] * (2 - nrx))
        ha = (_f32p * 8)(*[P(hs[p][a]) if a < nrx else None for p in range(4) for a in range(2)])
        r = f(nof_prb, cell_id, nports, nrx, ya, ha, noise, sf_idx, ctypes.byref(cfi), ctypes.byref(corr))
    elif ref:
        f = L.ref_pcfich
        f.argtypes = [ctypes.c_uint32] * 4 + [_f32p] * 6 + [ctypes.c_float, ctypes.c_uint32, _u32p,
                                                            _f32p, _u32p]
        g = lambda p, a: hs[p][a] if p < nports and a < nrx else None
        r = f(nof_prb, cell_id, nports, nrx, P(ys[0]), P(ys[1]) if nrx > 1 else None,
              P(g(0, 0)), P(g(0, 1)), P(g(1, 0)), P(g(1, 1)), noise, sf_idx, ctypes.byref(cfi),
              ctypes.byref(corr), None)
    else:
        f = L.orc_pcfich_decode
        f.argtypes = [ctypes.c_uint32] * 4 + [ctypes.POINTER(_f32p), ctypes.POINTER(_f32p),
                                              ctypes.c_float, ctypes.c_uint32, _u32p, _f32p]
        ya = (_f32p * 2)(*[P(v) for v in ys] + [None] * (2 - nrx))
        ha = (_f32p * 8)(*[P(hs[p][a]) for p in range(nports) for a in range(nrx)] +
                         [None] * (8 - nports * nrx))
        r = f(nof_prb, cell_id, nports, nrx, ya, ha, noise, sf_idx, ctypes.byref(cfi), ctypes.byref(corr))
    assert r == 0, r
    return cfi.value, corr.value


# ------------------------------------------------------------------ PDCCH / DCI ----
_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)


def _L(lib):
    return lib.lib if hasattr(lib, "lib") else lib


def _pf(a):
    return a.ctypes.data_as(_f32p) if a is not None else None


def pdcch_map(lib, nof_prb, cell_id, nports, phich_len, phich_res, cfi, ref=False):
    """srslte_regs_pdcch_get's symbol order as grid indices and NOF_CCE(cfi)"""
    f = getattr(_L(lib), "ref_pdcch_map" if ref else "orc_pdcch_map")
    f.argtypes = [ctypes.c_uint32] * 6 + [_u32p, _u32p]
    idx = np.zeros(4 * 3 * 110 * 4, np.uint32)
    ncce = ctypes.c_uint32(0)
    n = f(nof_prb, cell_id, nports, phich_len, phich_res, cfi, _ptr(idx, _u32p), ctypes.byref(ncce))
    assert n >= 0, n
    return idx[:n].copy(), ncce.value


def pdcch_encode(lib, nof_prb, cell_id, nports, phich_len, phich_res, cfi, sf_idx, msgs):
    """srslte_pdcch_encode of msgs [(bits, L, ncce, rnti)] -> port grids complex64 [nports][14 * 12 nof_prb]
    (reference build only). The reference cannot encode a message whose E = 72 * 2^L is not below
    q->max_bits = 72 NOF_CCE(3) (pdcch.c:548): srslte_pdcch_dci_encode then returns an error that
    srslte_pdcch_encode ignores, and uninitialised bits go out. Callers avoid such locations
    (pdcch_encodable); the result is checked to be finite."""
    f = _L(lib).ref_pdcch_encode if nports <= 2 else _L(lib).ref_pdcch_encode_n
    f.argtypes = [ctypes.c_uint32] * 8 + [_u8p, _u32p, _u32p, _u32p, _u16p] + (
        [_f32p, _f32p] if nports <= 2 else [ctypes.POINTER(_f32p)])
    n = 14 * 12 * nof_prb
    grids = [np.zeros(n, np.complex64) for _ in range(max(2, nports))]
    bits = np.zeros(128 * max(len(msgs), 1), np.uint8)
    nb = np.zeros(max(len(msgs), 1), np.uint32)
    Ls, nc = nb.copy(), nb.copy()
    rn = np.zeros(max(len(msgs), 1), np.uint16)
    for i, (b, L, c, r) in enumerate(msgs):
        bits[128 * i:128 * i + len(b)] = b
        nb[i], Ls[i], nc[i], rn[i] = len(b), L, c, r
    gp = [_pf(grids[0]), _pf(grids[1])] if nports <= 2 else [(_f32p * 4)(*[_pf(g) for g in grids])]
    assert f(nof_prb, cell_id, nports, phich_len, phich_res, cfi, sf_idx, len(msgs), _ptr(bits, _u8p),
             _ptr(nb, _u32p), _ptr(Ls, _u32p), _ptr(nc, _u32p), _ptr(rn, _u16p), *gp) == 0
    assert all(np.isfinite(g).all() for g in grids), "the reference PDCCH encoder sent uninitialised bits"
    return grids[:nports]


def pdcch_encodable(lib, nof_prb, cell_id, nports, phich_len, phich_res, L):
    """whether the reference's srslte_pdcch_encode can encode aggregation level L in this cell
    (72 * 2^L < q->max_bits = 72 NOF_CCE(3), pdcch.c:193, :548)"""
    return (1 << L) < pdcch_map(lib, nof_prb, cell_id, nports, phich_len, phich_res, 3, ref=True)[1]


def pdcch_llr(lib, nof_prb, cell_id, nports, phich_len, phich_res, nrx, cfi, sf_idx, noise, y, h, ref=False):
    """srslte_pdcch_extract_llr_multi: y[a] grids, h[p][a] estimates (complex64, 14 * 12 nof_prb or the
    leading control symbols, zero-padded) -> the 72 NOF_CCE(cfi) float LLRs"""
    n = 14 * 12 * nof_prb
    pad = lambda a: np.ascontiguousarray(np.concatenate([a, np.zeros(n - a.size, np.complex64)])
                                         if a.size < n else a, np.complex64)
    if nports == 4:
        f = getattr(_L(lib), "ref_pdcch_llr_n" if ref else "orc_pdcch_llr_n")
        f.argtypes = [ctypes.c_uint32] * 8 + [ctypes.c_float, ctypes.POINTER(_f32p), ctypes.POINTER(_f32p), _f32p]
        ys = [pad(y[a]) if a < nrx else None for a in range(2)]
        hs = [pad(h[p][a]) if a < nrx else None for p in range(4) for a in range(2)]
        llr = np.zeros(72 * 128, np.float32)
        e = f(nof_prb, cell_id, nports, phich_len, phich_res, nrx, cfi, sf_idx, noise,
              (_f32p * 2)(*[_pf(v) for v in ys]), (_f32p * 8)(*[_pf(v) for v in hs]), _pf(llr))
        assert e > 0, e
        return llr[:e].copy()
    f = getattr(_L(lib), "ref_pdcch_llr" if ref else "orc_pdcch_llr")
    f.argtypes = [ctypes.c_uint32] * 8 + [ctypes.c_float] + [_f32p] * 7
    ys = [pad(y[a]) if a < nrx else None for a in range(2)]
    hs = [[pad(h[p][a]) if p < nports and a < nrx else None for a in range(2)] for p in range(2)]
    llr = np.zeros(72 * 128, np.float32)  # NOF_CCE reaches 96 at 110 PRB
    e = f(nof_prb, cell_id, nports, phich_len, phich_res, nrx, cfi, sf_idx, noise, _pf(ys[0]), _pf(ys[1]),
          _pf(hs[0][0]), _pf(hs[0][1]), _pf(hs[1][0]), _pf(hs[1][1]), _pf(llr))
    assert e > 0, e
    return llr[:e].copy()


def find_dci(lib, nof_prb, cell_id, nports, phich_len, phich_res, cfi, sf_idx, llr, rnti, tm, rnti_type=-1,
             ul_rnti=0):
    """the oracle's srslte_ue_dl_find_dl_dci (rnti != 0) then srslte_ue_dl_find_ul_dci (ul_rnti != 0) on LLRs
    -> (dl, ul), each (found, format, L, ncce, nof_bits, buf): buf is the message buffer (128 bytes: the
    payload, then the 16 CRC bits) when found, else empty"""
    f = _L(lib).orc_find_dci
    f.argtypes = [ctypes.c_uint32] * 7 + [_f32p, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint16,
                                          _i32p, _u8p, _i32p, _u8p]
    llr = np.ascontiguousarray(llr, np.float32)
    o1, o2 = np.zeros(5, np.int32), np.zeros(5, np.int32)
    d1, d2 = np.zeros(128, np.uint8), np.zeros(128, np.uint8)
    assert f(nof_prb, cell_id, nports, phich_len, phich_res, cfi, sf_idx, _pf(llr), rnti, tm, rnti_type, ul_rnti,
             _ptr(o1, _i32p), _ptr(d1, _u8p), _ptr(o2, _i32p), _ptr(d2, _u8p)) == 0
    tup = lambda o, d: (int(o[0]), int(o[1]), int(o[2]), int(o[3]), int(o[4]), d.copy() if o[0] > 0 else d[:0].copy())
    return tup(o1, d1), tup(o2, d2)


def find_dl_dci(lib, nof_prb, cell_id, nports, phich_len, phich_res, cfi, sf_idx, llr, rnti, tm,
                rnti_type=-1, ref=False):
    """the oracle's srslte_ue_dl_find_dl_dci blind search on LLRs -> (found, format, L, ncce, nof_bits, buf).
    The reference's own search runs from grids: find_dci_ref."""
    assert not ref, "the reference search is ue_dl.c in oracle/_ref/ref_front: use find_dci_ref"
    return find_dci(lib, nof_prb, cell_id, nports, phich_len, phich_res, cfi, sf_idx, llr, rnti, tm, rnti_type)[0]


def find_dci_ref(nof_prb, cell_id, nports, nrx, phich_len, phich_res, cfi, sf_idx, noise, y, h, searches):
    """the reference's ue_dl.c (oracle/_ref/ref_front): srslte_pdcch_extract_llr_multi of y / h, then per
    search (rnti, tm, rnti_type, ul_rnti) srslte_ue_dl_find_dl_dci(_type) and srslte_ue_dl_find_ul_dci.
    -> (llr, [(dl, ul, ul_grant)]) with dl / ul as find_dci returns them"""
    sfs = [dict(sf_idx=sf_idx, cfi=cfi, noise=noise, rnti=r, tm=t, rnti_type=rt, ul_rnti=u, y=y, h=h)
           for r, t, rt, u in searches]
    res = ref_front_dci(nof_prb, cell_id, nports, nrx, phich_len, phich_res, sfs)
    for x in res:
        assert np.array_equal(x["llr"].view(np.uint32), res[0]["llr"].view(np.uint32))
    return res[0]["llr"], [(x["dl"], x["ul"], x["ul_grant"]) for x in res]


def dci_pack_ul_ref(lib, nof_prb, fields):
    """srslte_dci_msg_pack_pusch (format 0) of 8 fields (freq_hop_fl, L_crb, RB_start, mcs, ndi, tpc, n_dmrs,
    cqi_request) -> bits, or None"""
    f = _L(lib).ref_dci_pack_ul
    f.argtypes = [ctypes.c_uint32, _i32p, _u8p]
    fl = np.asarray(fields, np.int32)
    b = np.zeros(128, np.uint8)
    n = f(nof_prb, _ptr(fl, _i32p), _ptr(b, _u8p))
    return None if n < 0 else b[:n].copy()


def dci_to_ul_grant_ref(lib, bits, nof_prb, n_rb_ho=0, nof_bits=None):
    """srslte_dci_msg_to_ul_grant -> (ret, dci 11 fields, grant 10 fields) (ref_front.c's order)"""
    f = _L(lib).ref_dci_to_ul_grant
    f.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _i32p, _i32p]
    b = np.zeros(128, np.uint8)
    b[:len(bits)] = bits
    d, g = np.zeros(11, np.int32), np.zeros(10, np.int32)
    r = f(_ptr(b, _u8p), len(bits) if nof_bits is None else nof_bits, nof_prb, n_rb_ho, _ptr(d, _i32p),
          _ptr(g, _i32p))
    return r, d, g


def random_ul_msg(ref, rng, nof_prb, hop_p=0.2):
    """a format 0 DCI packed by the reference from random fields (hopping with probability hop_p)"""
    for _ in range(40):
        L = int(rng.integers(1, nof_prb + 1))
        hop = int(rng.integers(0, 4)) if rng.random() < hop_p else -1
        fields = [hop, L, int(rng.integers(0, nof_prb - L + 1)), int(rng.integers(0, 32)), int(rng.integers(0, 2)),
                  int(rng.integers(0, 4)), int(rng.integers(0, 8)), int(rng.integers(0, 2))]
        b = dci_pack_ul_ref(ref, nof_prb, fields)
        if b is not None:
            return b
    raise AssertionError("no format 0 message")


def pdcch_locations(lib, nof_cce, sf_idx, rnti, common, ref=True):
    f = getattr(_L(lib), "ref_pdcch_locations" if ref else "orc_pdcch_locations")
    f.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_int, _u32p]
    out = np.zeros(128, np.uint32)
    n = f(nof_cce, sf_idx, rnti, int(common), _ptr(out, _u32p))
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]


def dci_sizeof_ref(lib, fmt, nof_prb, nports):
    f = _L(lib).ref_dci_sizeof
    f.argtypes = [ctypes.c_uint32] * 3
    f.restype = ctypes.c_uint32
    return f(fmt, nof_prb, nports)


def dci_to_dl_grant_ref(lib, bits, fmt, rnti, nof_prb, nports, nof_bits=None):
    """srslte_dci_msg_to_dl_grant of the message bits[:nof_bits] (bits: the payload, or a 128-byte message
    buffer; zero-padded) -> (ret, dci 30 fields, grant 13 fields, prb_idx [2][110])"""
    f = _L(lib).ref_dci_to_dl_grant
    f.argtypes = [_u8p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32,
                  _i32p, _i32p, _u8p]
    b = np.zeros(128, np.uint8)
    b[:len(bits)] = bits
    nof_bits = len(bits) if nof_bits is None else nof_bits
    d, g, p = np.zeros(30, np.int32), np.zeros(13, np.int32), np.zeros(220, np.uint8)
    r = f(_ptr(b, _u8p), nof_bits, fmt, rnti, nof_prb, nports, _ptr(d, _i32p), _ptr(g, _i32p), _ptr(p, _u8p))
    return r, d, g, p.reshape(2, 110)


def dci_pack_dl_ref(lib, fmt, nof_prb, nports, crc_is_crnti, fields):
    """srslte_dci_msg_pack_pdsch from 30 fields -> bits, or None if the reference refuses them"""
    f = _L(lib).ref_dci_pack_dl
    f.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, _i32p, _u8p]
    fl = np.asarray(fields, np.int32)
    b = np.zeros(128, np.uint8)
    n = f(fmt, nof_prb, nports, int(crc_is_crnti), _ptr(fl, _i32p), _ptr(b, _u8p))
    return None if n < 0 else b[:n].copy()


# srslte_dci_format_t
F0, F1, F1A, F1C, F1B, F1D, F2, F2A, F2B = range(9)
UE_FORMATS = [(F1A, F1), (F1A, F1), (F1A, F2A), (F1A, F2), (F1A, F1D), (F1A, F1B), (F1A, F1), (F1A, F2B)]


def random_dl_fields(rng, fmt, nof_prb):
    """random srslte_ra_dl_dci_t fields (30, ref_harness order) that dci.c's packers mostly accept"""
    f = [0] * 30
    P = 1 if nof_prb <= 10 else 2 if nof_prb <= 26 else 3 if nof_prb <= 63 else 4
    asz = -(-nof_prb // P)
    if fmt in (F1, F2, F2A, F2B):
        f[0] = int(rng.integers(0, 2)) if nof_prb > 10 else 0
        if f[0] == 0:
            f[1] = int(rng.integers(0, 1 << asz))
        else:
            lp = int(np.ceil(np.log2(P)))
            f[3], f[4] = int(rng.integers(0, P)), int(rng.integers(0, 2))
            f[2] = int(rng.integers(0, 1 << max(asz - lp - 1, 0)))
    else:
        f[0] = 2
        f[10] = 1 if fmt == F1C else int(rng.integers(0, 2))
        f[9] = int(rng.integers(0, 2)) if nof_prb >= 50 else 0
        step = 2 if nof_prb < 50 else 4
        lim = nof_prb if f[10] == 0 else min(nof_prb, 16 if nof_prb > 50 else nof_prb)
        if fmt == F1C:
            L = step * int(rng.integers(1, max(lim // step, 1) + 1))
            f[6], f[7] = L, step * int(rng.integers(0, max((lim - L) // step, 0) + 1))
        else:
            L = int(rng.integers(1, lim + 1))
            f[6], f[7] = L, int(rng.integers(0, lim - L + 1))
        f[8] = int(rng.integers(0, 2))
    f[11] = int(rng.integers(0, 8))
    f[12] = int(rng.integers(0, 32)) if rng.random() < 0.15 else int(rng.integers(0, 29))
    f[13], f[14] = int(rng.integers(0, 4)), int(rng.integers(0, 2))
    f[15], f[16], f[17] = int(rng.integers(0, 29)), int(rng.integers(0, 4)), int(rng.integers(0, 2))
    f[18], f[19] = int(rng.integers(0, 2)), int(rng.integers(0, 2))
    f[20] = int(rng.integers(0, 8))
    f[23] = 1
    f[24] = int(rng.integers(0, 2)) if fmt in (F2, F2A, F2B) else 0
    return f


def random_dl_msg(ref, rng, fmt, nof_prb, nports, crc_is_crnti=True, tries=40):
    """a DCI message of format fmt: packed by the reference from random fields where dci.c packs the
    format (1, 1A, 1C, 2, 2A, 2B), else (or if every try is refused) random bits of the format's size"""
    if fmt in (F1, F1A, F1C, F2, F2A, F2B):
        for _ in range(tries):
            b = dci_pack_dl_ref(ref, fmt, nof_prb, nports, crc_is_crnti, random_dl_fields(rng, fmt, nof_prb))
            if b is not None:
                return b
    n = dci_sizeof_ref(ref, fmt, nof_prb, nports)
    b = rng.integers(0, 2, n).astype(np.uint8)
    if fmt == F1A:
        b[0] = 1
    return b


def pdcch_subframe(ref, rng, nof_prb, cell_id, nports, nrx, phich_len, phich_res, cfi, sf_idx, tm,
                   snr_db=12.0):
    """A synthetic received control region built with the reference's srslte_pdcch_encode: DCIs for a
    C-RNTI in its UE-specific space (the tm's formats, sometimes a format 0 look-alike before it) and
    for SI- / RA-RNTIs in the common space, through a flat per-(port, antenna) channel with small
    per-RE ripple and AWGN. Returns (y[nrx], h[nports][nrx] over the 4 leading symbols, searches
    [(rnti, tm, rnti_type, ul_rnti)], noise estimate)."""
    idx, ncce = pdcch_map(ref, nof_prb, cell_id, nports, phich_len, phich_res, cfi, ref=True)
    used = np.zeros(max(ncce, 1), bool)
    msgs = []

    ncce3 = pdcch_map(ref, nof_prb, cell_id, nports, phich_len, phich_res, 3, ref=True)[1]

    def place(locs, bits, rnti):
        rng.shuffle(locs)
        for L, c in locs:
            # srslte_dci_location_isvalid, and a level the reference's encoder can encode (pdcch_encode)
            if c <= 87 and (1 << L) < ncce3 and not used[c:c + (1 << L)].any():
                used[c:c + (1 << L)] = True
                msgs.append((bits, L, c, rnti))
                return True
        return False

    crnti = int(rng.integers(0x000B, 0xFFF4))
    ue = pdcch_locations(ref, ncce, sf_idx, crnti, False)
    com = pdcch_locations(ref, ncce, sf_idx, 0, True)
    if ue and rng.random() < 0.4:  # a UL grant (format 0 shares 1A's size): the DL search sets it aside
        if rng.random() < 0.5:
            b = random_ul_msg(ref, rng, nof_prb)
        else:
            b = rng.integers(0, 2, dci_sizeof_ref(ref, F0, nof_prb, nports)).astype(np.uint8)
            b[0] = 0
        place(list(ue), b, crnti)
    if ue and rng.random() < 0.9:
        fmt = UE_FORMATS[tm][int(rng.integers(0, 2))]
        place(list(ue), random_dl_msg(ref, rng, fmt, nof_prb, nports), crnti)
    elif com:
        place(list(com), random_dl_msg(ref, rng, F1A, nof_prb, nports), crnti)
    si = 0xFFFF
    if com and rng.random() < 0.8:
        fmt = F1A if rng.random() < 0.5 else F1C
        place(list(com), random_dl_msg(ref, rng, fmt, nof_prb, nports, crc_is_crnti=False), si)
    rarnti = int(rng.integers(1, 11))
    if com and rng.random() < 0.5:
        place(list(com), random_dl_msg(ref, rng, F1A, nof_prb, nports, crc_is_crnti=False), rarnti)
    x = pdcch_encode(ref, nof_prb, cell_id, nports, phich_len, phich_res, cfi, sf_idx, msgs)
    n4 = 4 * 12 * nof_prb
    sigma = 10 ** (-snr_db / 20) / np.sqrt(2)
    h = [[None] * nrx for _ in range(nports)]
    y = []
    for a in range(nrx):
        acc = np.zeros(n4, np.complex64)
        for p in range(nports):
            g = np.exp(2j * np.pi * rng.random()) * (0.8 + 0.4 * rng.random())
            ripple = 1 + 0.05 * (rng.standard_normal(n4) + 1j * rng.standard_normal(n4))
            h[p][a] = (g * ripple).astype(np.complex64)
            acc += h[p][a] * x[p][:n4]
        acc += (sigma * (rng.standard_normal(n4) + 1j * rng.standard_normal(n4))).astype(np.complex64)
        y.append(acc.astype(np.complex64))
    # (DL rnti, tm, rnti_type, UL rnti): phch_worker's DL search, then its UL search for the C-RNTI
    searches = [(crnti, tm, -1, crnti), (si, tm, -1, crnti), (rarnti, tm, -1, 0),
                (int(rng.integers(0x000B, 0xFFF4)), tm, -1, crnti), (si, tm, 1, 0), (crnti, tm, 0, crnti),
                (crnti, tm, -1, 0)]
    noise = float(2 * sigma * sigma) if rng.random() < 0.7 else 0.0
    return y, h, searches, noise
