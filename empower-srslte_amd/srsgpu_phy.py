"""Python host-side mirror of the srsLTE turbo-decoder API on the MI355X engine.

Loads lib/libsrsgpu_phy.so (built by `make -C empower-srslte_amd`, C ABI in
include/srslte/phy/fec/turbodecoder.h and include/srsgpu/tdec_batch.h) through ctypes.

  Tdec       one srslte_tdec_t object (reference: lib/src/phy/fec/turbodecoder.c:133-564):
             init/new_cb/iteration/run_all/get_nof_iterations/free, same return codes.
  TdecBatch  the batched extension: many code blocks of one size per call, host arrays or
             device pointers (e.g. torch.cuda tensors' data_ptr()).

There is no CPU fallback: if the library is missing this module raises at import time.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SRSGPU_LIB") or os.path.join(_HERE, "lib", "libsrsgpu_phy.so")  # debug builds

SRSLTE_TDEC_AUTO, SRSLTE_TDEC_GENERIC, SRSLTE_TDEC_SSE = 0, 1, 2
SRSLTE_TDEC_SSE_WINDOW, SRSLTE_TDEC_AVX_WINDOW = 3, 4
SRSLTE_TDEC_SSE8_WINDOW, SRSLTE_TDEC_AVX8_WINDOW = 5, 6
SRSGPU_TDEC_AUTO_8BIT = 16  # include/srsgpu/tdec_batch.h: the reference's 8-bit AUTO path
SRSLTE_TDEC_SSE8_WINDOW, SRSLTE_TDEC_AVX8_WINDOW = 5, 6
SRSLTE_SUCCESS, SRSLTE_ERROR = 0, -1
CRC24A, CRC24B = 0x1864CFB, 0x1800063

try:
    # One HIP runtime per process: torch wheels bundle their own libamdhip64/libhsa-runtime64
    # with the same SONAME as /opt/rocm's. Loading torch first makes the library bind to that
    # runtime; loading the library first would put two HSA runtimes in the process and torch
    # then sees no GPU.
    import torch  # noqa: F401
except ImportError:  # C-only users: the library uses the system ROCm runtime
    torch = None

if not os.path.exists(LIB_PATH):
    raise ImportError("srsgpu: %s not found — build it with `make -C empower-srslte_amd` "
                      "(no CPU fallback exists)" % LIB_PATH)

_lib = ctypes.CDLL(LIB_PATH)
_vp, _sz, _u32, _i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
_i16p = ctypes.POINTER(ctypes.c_int16)
_i8p = ctypes.POINTER(ctypes.c_int8)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)


SRSLTE_TDEC_REF_SIZEOF = 18264  # include/srslte/phy/fec/turbodecoder.h: the reference's sizeof


class srslte_tdec_t(ctypes.Structure):
    """Layout of srslte_tdec_t in include/srslte/phy/fec/turbodecoder.h, padding included (the
    library clears and writes the whole struct)."""
    _fields_ = [("max_long_cb", ctypes.c_uint32), ("dec_type", ctypes.c_int),
                ("force_not_sb", ctypes.c_bool), ("current_long_cb", ctypes.c_uint32),
                ("current_cbidx", ctypes.c_int), ("n_iter", ctypes.c_int), ("gpu", ctypes.c_void_p),
                ("reserved", ctypes.c_uint8 * (SRSLTE_TDEC_REF_SIZEOF - 32))]


assert ctypes.sizeof(srslte_tdec_t) == SRSLTE_TDEC_REF_SIZEOF


class srslte_tcod_t(ctypes.Structure):
    """Layout of srslte_tcod_t in include/srslte/phy/fec/turbocoder.h."""
    _fields_ = [("max_long_cb", ctypes.c_uint32), ("temp", ctypes.c_void_p)]


class srsgpu_dlsch_tb_t(ctypes.Structure):
    """include/srsgpu/dlsch_batch.h"""
    _fields_ = [("tbs", ctypes.c_uint32), ("rv", ctypes.c_uint32), ("Qm", ctypes.c_uint32),
                ("nof_e_bits", ctypes.c_uint32), ("softbuffer", ctypes.c_uint32),
                ("e_offset", ctypes.c_uint64), ("data_offset", ctypes.c_uint64)]


class srsgpu_ulsch_tb_t(ctypes.Structure):
    """include/srsgpu/ulsch_batch.h"""
    _fields_ = [("tbs", ctypes.c_uint32), ("rv", ctypes.c_uint32), ("Qm", ctypes.c_uint32),
                ("nof_bits", ctypes.c_uint32), ("nof_symb", ctypes.c_uint32),
                ("softbuffer", ctypes.c_uint32), ("q_offset", ctypes.c_uint64),
                ("data_offset", ctypes.c_uint64)]


UCI_MAX_CQI_BITS = 183


class srsgpu_uci_cfg_t(ctypes.Structure):
    """include/srsgpu/ulsch_batch.h"""
    _fields_ = [(n, ctypes.c_uint32) for n in ("O_ack", "O_ri", "O_cqi", "I_offset_ack", "I_offset_ri",
                                                 "I_offset_cqi", "M_sc", "M_sc_init")] + [("c_offset", ctypes.c_uint64)]


class srsgpu_uci_result_t(ctypes.Structure):
    """include/srsgpu/ulsch_batch.h"""
    _fields_ = [("ack", ctypes.c_uint8 * 2), ("ri", ctypes.c_uint8), ("cqi_ack", ctypes.c_uint8),
                ("cqi", ctypes.c_uint8 * (UCI_MAX_CQI_BITS + 1)), ("Q_ack", ctypes.c_uint32),
                ("Q_ri", ctypes.c_uint32), ("Q_cqi", ctypes.c_uint32)]


SOFTBUFFER_SIZE = 18600


class srsgpu_cell_t(ctypes.Structure):
    """include/srsgpu/pdsch_batch.h"""
    _fields_ = [("nof_prb", ctypes.c_uint32), ("id", ctypes.c_uint32),
                ("nof_ports", ctypes.c_uint32), ("nof_rx_ant", ctypes.c_uint32), ("cp", ctypes.c_uint32)]


MIMO_SINGLE_ANTENNA, MIMO_TX_DIVERSITY, MIMO_SPATIAL_MULTIPLEX, MIMO_CDD = 0, 1, 2, 3


class srsgpu_pdsch_sf_t(ctypes.Structure):
    """include/srsgpu/pdsch_batch.h"""
    _fields_ = [("sf_idx", ctypes.c_uint32), ("lstart", ctypes.c_uint32),
                ("prb_idx", (ctypes.c_uint8 * 110) * 2), ("nof_re", ctypes.c_uint32),
                ("rnti", ctypes.c_uint16), ("noise_estimate", ctypes.c_float),
                ("scaling", ctypes.c_float), ("mimo_type", ctypes.c_uint32),
                ("tb_cw_swap", ctypes.c_uint32), ("mod", ctypes.c_uint32 * 2),
                ("tbs", ctypes.c_uint32 * 2), ("rv", ctypes.c_uint32 * 2),
                ("softbuffer", ctypes.c_uint32 * 2), ("grid_offset", ctypes.c_uint64),
                ("ce_offset", ctypes.c_uint64), ("data_offset", ctypes.c_uint64 * 2),
                ("codebook_idx", ctypes.c_uint32), ("skip_tb", ctypes.c_uint32)]


class srsgpu_rxq_meas_t(ctypes.Structure):
    """include/srsgpu/rx_queue.h: srslte_chest_dl_get_* of a subframe"""
    _fields_ = [("cfo", ctypes.c_float), ("snr", ctypes.c_float), ("rsrp", ctypes.c_float), ("rsrq", ctypes.c_float),
                ("rssi", ctypes.c_float), ("rsrp_neighbour", ctypes.c_float)]

    def values(self):
        return [self.cfo, self.snr, self.rsrp, self.rsrq, self.rssi, self.rsrp_neighbour]


class srsgpu_feedback_sf_t(ctypes.Structure):
    """include/srsgpu/pdsch_batch.h"""
    _fields_ = [("ce_offset", ctypes.c_uint64), ("noise_estimate", ctypes.c_float), ("flags", ctypes.c_uint32)]


class srsgpu_feedback_t(ctypes.Structure):
    """include/srsgpu/pdsch_batch.h: TM3 / TM4 feedback of a subframe"""
    _fields_ = [("cn", ctypes.c_float), ("ri_tm3", ctypes.c_uint32), ("ret_cn", ctypes.c_int32),
                ("ri", ctypes.c_uint32), ("pmi", ctypes.c_uint32), ("pmi_l", ctypes.c_uint32 * 2),
                ("ret_pmi", ctypes.c_int32), ("sinr", (ctypes.c_float * 4) * 2)]

    def sinr_array(self):
        import numpy as np
        return np.array([[self.sinr[l][c] for c in range(4)] for l in range(2)], np.float32)


FEEDBACK_CN, FEEDBACK_PMI = 1, 2


class srsgpu_rxq_item_t(ctypes.Structure):
    """include/srsgpu/rx_queue.h"""
    _fields_ = [("td", ctypes.c_void_p * 2), ("sf", srsgpu_pdsch_sf_t),
                ("reset_softbuffer", ctypes.c_uint32 * 2), ("data", ctypes.c_void_p * 2),
                ("ret", ctypes.c_int32 * 2), ("noi", ctypes.c_uint32 * 2), ("noise", ctypes.c_float),
                ("meas", srsgpu_rxq_meas_t)]


class srsgpu_viterbi_frame_t(ctypes.Structure):
    """include/srsgpu/viterbi_batch.h"""
    _fields_ = [("sym_offset", ctypes.c_uint64), ("out_offset", ctypes.c_uint64),
                ("frame_length", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class srsgpu_dci_cand_t(ctypes.Structure):
    """include/srsgpu/viterbi_batch.h"""
    _fields_ = [("llr_offset", ctypes.c_uint64), ("out_offset", ctypes.c_uint64),
                ("E", ctypes.c_uint32), ("nof_bits", ctypes.c_uint32)]


class srsgpu_pcfich_sf_t(ctypes.Structure):
    """include/srsgpu/pcfich_batch.h"""
    _fields_ = [("grid_offset", ctypes.c_uint64), ("ce_offset", ctypes.c_uint64),
                ("sf_idx", ctypes.c_uint32), ("noise_estimate", ctypes.c_float)]


class srsgpu_pdcch_sf_t(ctypes.Structure):
    """include/srsgpu/pdcch_batch.h"""
    _fields_ = [("grid_offset", ctypes.c_uint64), ("ce_offset", ctypes.c_uint64),
                ("llr_offset", ctypes.c_uint64), ("sf_idx", ctypes.c_uint32), ("cfi", ctypes.c_uint32),
                ("noise_estimate", ctypes.c_float), ("reserved", ctypes.c_uint32)]


class srsgpu_dci_location_t(ctypes.Structure):
    """include/srsgpu/pdcch_batch.h"""
    _fields_ = [("L", ctypes.c_uint32), ("ncce", ctypes.c_uint32)]


class srsgpu_dci_search_t(ctypes.Structure):
    """include/srsgpu/pdcch_batch.h"""
    _fields_ = [("llr_offset", ctypes.c_uint64), ("sf_idx", ctypes.c_uint32), ("cfi", ctypes.c_uint32),
                ("rnti", ctypes.c_uint32), ("tm", ctypes.c_uint32), ("rnti_type", ctypes.c_int32),
                ("ul_rnti", ctypes.c_uint32)]


class srsgpu_dci_result_t(ctypes.Structure):
    """include/srsgpu/pdcch_batch.h"""
    _fields_ = [("found", ctypes.c_int32), ("format", ctypes.c_uint32), ("L", ctypes.c_uint32),
                ("ncce", ctypes.c_uint32), ("nof_bits", ctypes.c_uint32), ("data", ctypes.c_uint8 * 128)]


DCI_FORMAT0, DCI_FORMAT1, DCI_FORMAT1A, DCI_FORMAT1C, DCI_FORMAT1B, DCI_FORMAT1D = range(6)
DCI_FORMAT2, DCI_FORMAT2A, DCI_FORMAT2B = 6, 7, 8


class srsgpu_ra_dl_dci_t(ctypes.Structure):
    """include/srsgpu/dci.h"""
    _fields_ = [(n, ctypes.c_uint32) for n in ("alloc_type", "rbg_bitmask", "vrb_bitmask", "rbg_subset",
                                               "shift", "riv", "L_crb", "RB_start", "n_prb1a", "n_gap",
                                               "mode", "harq_process", "mcs_idx")] + \
        [("rv_idx", ctypes.c_int32), ("ndi", ctypes.c_uint32), ("mcs_idx_1", ctypes.c_uint32),
         ("rv_idx_1", ctypes.c_int32)] + \
        [(n, ctypes.c_uint32) for n in ("ndi_1", "tb_cw_swap", "sram_id", "pinfo", "pconf", "power_offset")] + \
        [("tb_en", ctypes.c_uint32 * 2)] + \
        [(n, ctypes.c_uint32) for n in ("is_ra_order", "ra_preamble", "ra_mask_idx", "dci_is_1a", "dci_is_1c")]
    # the reference harness's 30-field order (oracle/ref_harness.c ref_dci_out)
    ORDER = ("alloc_type", "rbg_bitmask", "vrb_bitmask", "rbg_subset", "shift", "riv", "L_crb", "RB_start",
             "n_prb1a", "n_gap", "mode", "harq_process", "mcs_idx", "rv_idx", "ndi", "mcs_idx_1", "rv_idx_1",
             "ndi_1", "tb_cw_swap", "sram_id", "pinfo", "pconf", "power_offset", "tb_en0", "tb_en1",
             "is_ra_order", "ra_preamble", "ra_mask_idx", "dci_is_1a", "dci_is_1c")

    def fields30(self):
        return [self.tb_en[int(n[-1])] if n.startswith("tb_en") else getattr(self, n) for n in self.ORDER]


class srsgpu_ra_dl_grant_t(ctypes.Structure):
    """include/srsgpu/dci.h"""
    _fields_ = [("prb_idx", (ctypes.c_uint8 * 110) * 2), ("nof_prb", ctypes.c_uint32),
                ("Qm", ctypes.c_uint32 * 2), ("mod", ctypes.c_uint32 * 2), ("tbs", ctypes.c_int32 * 2),
                ("mcs_idx", ctypes.c_uint32 * 2), ("tb_en", ctypes.c_uint32 * 2), ("pinfo", ctypes.c_uint32),
                ("tb_cw_swap", ctypes.c_uint32)]

    def fields13(self):
        """the reference harness's 13-field order (oracle/ref_harness.c ref_dci_to_dl_grant)"""
        return [self.nof_prb, self.Qm[0], self.Qm[1], self.mod[0], self.tbs[0], self.mcs_idx[0], self.mod[1],
                self.tbs[1], self.mcs_idx[1], self.tb_en[0], self.tb_en[1], self.pinfo, self.tb_cw_swap]


class srsgpu_ra_ul_dci_t(ctypes.Structure):
    """include/srsgpu/dci.h (format 0)"""
    _fields_ = [("freq_hop_fl", ctypes.c_int32)] + [(n, ctypes.c_uint32) for n in (
        "riv", "L_crb", "RB_start", "mcs_idx", "rv_idx", "n_dmrs", "ndi", "cqi_request", "tpc_pusch")]

    def fields11(self):
        """oracle/ref_front.c's order"""
        return [self.freq_hop_fl, self.riv, self.L_crb, self.RB_start, self.mcs_idx, self.rv_idx, self.n_dmrs,
                self.ndi, self.cqi_request, self.tpc_pusch, 0]


class srsgpu_ra_ul_grant_t(ctypes.Structure):
    """include/srsgpu/dci.h"""
    _fields_ = [("L_prb", ctypes.c_uint32), ("n_prb", ctypes.c_uint32 * 2)] + \
        [(n, ctypes.c_uint32) for n in ("freq_hopping", "M_sc", "M_sc_init", "Qm", "mod")] + \
        [("tbs", ctypes.c_int32), ("mcs_idx", ctypes.c_uint32), ("ncs_dmrs", ctypes.c_uint32)]

    def fields10(self):
        """oracle/ref_front.c's order"""
        return [self.L_prb, self.n_prb[0], self.n_prb[1], self.freq_hopping, self.M_sc, self.Qm, self.mod, self.tbs,
                self.mcs_idx, self.ncs_dmrs]


class srsgpu_rxq_ue_dl_t(ctypes.Structure):
    """include/srsgpu/rx_queue.h: one srslte_ue_dl_decode_rnti subframe"""
    _fields_ = [("td", ctypes.c_void_p * 2), ("tti", ctypes.c_uint32), ("rnti", ctypes.c_uint16),
                ("tm", ctypes.c_uint32), ("rnti_type", ctypes.c_int32), ("softbuffer", ctypes.c_uint32 * 2),
                ("data", ctypes.c_void_p * 2), ("acks", ctypes.c_uint8 * 2), ("ret", ctypes.c_int32),
                ("cfi", ctypes.c_uint32), ("cfi_corr", ctypes.c_float), ("found", ctypes.c_int32),
                ("format", ctypes.c_uint32), ("L", ctypes.c_uint32), ("ncce", ctypes.c_uint32),
                ("mimo_type", ctypes.c_uint32), ("rv", ctypes.c_uint32 * 2), ("grant", srsgpu_ra_dl_grant_t),
                ("noi", ctypes.c_uint32 * 2), ("noise", ctypes.c_float),
                ("ul_rnti", ctypes.c_uint16), ("n_rb_ho", ctypes.c_uint32), ("ul_found", ctypes.c_int32),
                ("ul_L", ctypes.c_uint32), ("ul_ncce", ctypes.c_uint32), ("ul_nof_bits", ctypes.c_uint32),
                ("ul_data", ctypes.c_uint8 * 128), ("ul_grant_ret", ctypes.c_int32), ("ul_dci", srsgpu_ra_ul_dci_t),
                ("ul_grant", srsgpu_ra_ul_grant_t), ("acked_in", ctypes.c_uint8 * 2),
                ("dci_nof_bits", ctypes.c_uint32), ("dci_data", ctypes.c_uint8 * 128), ("meas", srsgpu_rxq_meas_t),
                ("feedback", ctypes.c_uint32), ("fb", srsgpu_feedback_t)]

    def dci_bits(self):
        return list(self.dci_data[:self.dci_nof_bits])


def dlsch_data_len(tbs):
    return tbs // 8 + 6


_P = ctypes.POINTER(srslte_tdec_t)
_PC = ctypes.POINTER(srslte_tcod_t)
_sig = {
    "srslte_tdec_init": (_i32, [_P, _u32]),
    "srslte_tdec_init_manual": (_i32, [_P, _u32, _i32]),
    "srslte_tdec_free": (None, [_P]),
    "srslte_tdec_force_not_sb": (None, [_P]),
    "srslte_tdec_new_cb": (_i32, [_P, _u32]),
    "srslte_tdec_get_nof_iterations": (_i32, [_P]),
    "srslte_tdec_autoimp_get_subblocks": (_u32, [_u32]),
    "srslte_tdec_autoimp_get_subblocks_8bit": (_u32, [_u32]),
    "srslte_tdec_iteration": (None, [_P, _i16p, _u8p]),
    "srslte_tdec_run_all": (_i32, [_P, _i16p, _u8p, _u32, _u32]),
    "srslte_tdec_iteration_8bit": (None, [_P, _i8p, _u8p]),
    "srslte_tdec_run_all_8bit": (_i32, [_P, _i8p, _u8p, _u32, _u32]),
    "srslte_tcod_init": (_i32, [_PC, _u32]),
    "srslte_tcod_free": (None, [_PC]),
    "srslte_tcod_encode": (_i32, [_PC, _u8p, _u8p, _u32]),
    "srsgpu_tdec_batch_create": (_i32, [ctypes.POINTER(_vp), _u32, _u32]),
    "srsgpu_tdec_batch_destroy": (None, [_vp]),
    "srsgpu_tdec_batch_set_stream": (None, [_vp, _vp]),
    "srsgpu_tdec_batch_run_dev": (_i32, [_vp, _i32, _i32, _vp, _sz, _u32, _u32, _u32, _vp, _sz]),
    "srsgpu_tdec_batch_decode_dev": (_i32, [_vp, _i32, _i32, _vp, _sz, _u32, _u32, _u32, _u32,
                                            _u32, _vp, _sz, _vp, _vp]),
    "srsgpu_tdec_batch_run": (_i32, [_vp, _i32, _i32, ctypes.POINTER(_vp), _u32, _u32, _u32,
                                     ctypes.POINTER(_vp)]),
    "srsgpu_tdec_batch_decode": (_i32, [_vp, _i32, _i32, ctypes.POINTER(_vp), _u32, _u32, _u32,
                                        _u32, _u32, ctypes.POINTER(_vp), _u8p, _u32p]),
    "srsgpu_tdec_input_len": (_u32, [_i32, _i32, _u32]),
    "srsgpu_tdec_batch_read_state": (_i32, [_vp, _u32, _i16p, _i16p]),
    "srsgpu_dlsch_create": (_i32, [ctypes.POINTER(_vp), _u32, _u32, _u32]),
    "srsgpu_dlsch_destroy": (None, [_vp]),
    "srsgpu_dlsch_set_stream": (None, [_vp, _vp]),
    "srsgpu_dlsch_softbuffer_reset": (_i32, [_vp, _u32]),
    "srsgpu_dlsch_softbuffer_reset_tbs": (_i32, [_vp, _u32, _u32]),
    "srsgpu_dlsch_softbuffer_reset_range": (_i32, [_vp, _u32, _u32]),
    "srsgpu_ulsch_deinterleave_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_ulsch_tb_t), _u32, _vp, _vp]),
    "srsgpu_ulsch_decode_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_ulsch_tb_t), _u32, _vp, _vp, _vp, _u32,
                                       _vp, _vp]),
    "srsgpu_ulsch_uci_decode_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_ulsch_tb_t), ctypes.POINTER(srsgpu_uci_cfg_t),
                                           _u32, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp]),
    "srsgpu_dlsch_decode_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_dlsch_tb_t), _u32, _vp, _vp, _u32,
                                       _vp, _vp]),
    "srsgpu_dlsch_decode": (_i32, [_vp, ctypes.POINTER(srsgpu_dlsch_tb_t), _u32,
                                   ctypes.POINTER(_vp), ctypes.POINTER(_vp), _u32,
                                   ctypes.POINTER(ctypes.c_int32), _u32p]),
    "srsgpu_dlsch_softbuffer_read": (_i32, [_vp, _u32, _i16p, _u8p]),
    "srsgpu_shard_contiguous": (_i32, [_u32, _u32, _u32p]),
    "srsgpu_shard_weighted": (_i32, [ctypes.POINTER(ctypes.c_uint64), _u32, _u32,
                                     ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_uint64)]),
    "srsgpu_rm_turbo_rx_dev": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32, _i32]),
    "srsgpu_dlsch_encode_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_dlsch_tb_t), _u32, _vp, _vp]),
    "srsgpu_pdsch_create": (_i32, [ctypes.POINTER(_vp), ctypes.POINTER(srsgpu_cell_t), _u32, _u32,
                                   _u32]),
    "srsgpu_pdsch_destroy": (None, [_vp]),
    "srsgpu_pdsch_set_stream": (None, [_vp, _vp]),
    "srsgpu_pdsch_set_csi": (None, [_vp, _i32]),
    "srsgpu_pdsch_set_llr_8bit": (None, [_vp, _i32]),
    "srsgpu_pdsch_set_ce_rows": (_i32, [_vp, _i32]),
    "srsgpu_chest_set_ce_rows": (None, [_vp, _i32]),
    "srsgpu_viterbi37_tb_decode_f_dev": (_i32, [_vp, _u32, _vp, _vp, _vp]),
    "srsgpu_dci_decode_dev": (_i32, [_vp, _u32, _vp, _vp, _vp, _vp, _vp]),
    "srsgpu_pcfich_create": (_i32, [ctypes.POINTER(_vp), ctypes.POINTER(srsgpu_cell_t)]),
    "srsgpu_pcfich_destroy": (None, [_vp]),
    "srsgpu_pcfich_re_map": (_i32, [_vp, _u32p]),
    "srsgpu_pcfich_set_noise_dev": (None, [_vp, _vp]),
    "srsgpu_pdcch_set_noise_dev": (None, [_vp, _vp]),
    "srsgpu_pcfich_decode_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_pcfich_sf_t), _u32, _vp, _vp, _sz,
                                        _vp, _vp, _vp]),
    "srsgpu_pdcch_create": (_i32, [ctypes.POINTER(_vp), ctypes.POINTER(srsgpu_cell_t), _u32, _u32]),
    "srsgpu_pdcch_destroy": (None, [_vp]),
    "srsgpu_pdcch_cell_map": (_i32, [ctypes.POINTER(srsgpu_cell_t), _u32, _u32, _u32, _u32p, _u32, _u32p]),
    "srsgpu_pdcch_nof_cce": (_u32, [_vp, _u32]),
    "srsgpu_pdcch_re_map": (_i32, [_vp, _u32, _u32p, _u32]),
    "srsgpu_pdcch_extract_llr_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_pdcch_sf_t), _u32, _vp, _vp, _sz, _vp,
                                            _vp]),
    "srsgpu_pdcch_ue_locations": (_u32, [_u32, _u32, ctypes.c_uint16, ctypes.POINTER(srsgpu_dci_location_t),
                                         _u32]),
    "srsgpu_pdcch_common_locations": (_u32, [_u32, ctypes.POINTER(srsgpu_dci_location_t), _u32]),
    "srsgpu_pdcch_find_dl_dci_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_dci_search_t), _u32, _vp, _vp, _vp]),
    "srsgpu_pdcch_find_dci_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_dci_search_t), _u32, _vp, _vp, _vp, _vp]),
    "srsgpu_dci_msg_to_ul_grant": (_i32, [_u8p, _u32, _u32, _u32, ctypes.POINTER(srsgpu_ra_ul_dci_t),
                                          ctypes.POINTER(srsgpu_ra_ul_grant_t)]),
    "srsgpu_dci_format_sizeof": (_u32, [_u32, _u32, _u32]),
    "srsgpu_dci_msg_to_dl_grant": (_i32, [_u8p, _u32, _u32, ctypes.c_uint16, _u32, _u32,
                                          ctypes.POINTER(srsgpu_ra_dl_dci_t),
                                          ctypes.POINTER(srsgpu_ra_dl_grant_t)]),
    "srsgpu_ra_dl_dci_to_grant": (_i32, [ctypes.POINTER(srsgpu_ra_dl_dci_t), _u32, ctypes.c_uint16,
                                         ctypes.POINTER(srsgpu_ra_dl_grant_t)]),
    "srsgpu_ra_tbs_from_idx": (_i32, [_u32, _u32]),
    "srsgpu_ra_tbs_idx_from_mcs": (_i32, [_u32]),
    "srsgpu_rxq_create": (_i32, [ctypes.POINTER(_vp), _vp, _u32, _u32, _u32, _u32, _u32]),
    "srsgpu_rxq_destroy": (None, [_vp]),
    "srsgpu_rxq_submit": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64)]),
    "srsgpu_rxq_wait": (_i32, [_vp, ctypes.c_uint64]),
    "srsgpu_rxq_decode": (_i32, [_vp, _vp]),
    "srsgpu_rxq_flush": (None, [_vp]),
    "srsgpu_rxq_stats": (None, [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "srsgpu_rxq_timing": (None, [_vp, ctypes.POINTER(ctypes.c_double), _u32]),
    "srsgpu_dlsch_softbuffer_reset_list": (_i32, [_vp, _u32p, _u32p, _u32]),
    "srsgpu_tdec_set_schedule": (ctypes.c_int, [ctypes.c_int] * 4),
    "srsgpu_tdec_get_schedule": (None, [ctypes.POINTER(ctypes.c_int)] * 4),
    "srsgpu_knobs_reload": (None, []),
    "srsgpu_rxq_drive": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32, _vp, _vp, _vp]),
    "srsgpu_rxq_drive_paced": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_void_p)] + [ctypes.c_uint32] * 5 +
                               [_vp, _vp, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_double)]),
    "srsgpu_rxq_register": (_i32, [_vp, _vp, ctypes.c_size_t]),
    "srsgpu_rxq_unregister": (_i32, [_vp, _vp]),
    "srsgpu_rxq_alloc_host": (_vp, [_vp, ctypes.c_size_t]),
    "srsgpu_rxq_drive_paced_ex": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_void_p)] + [ctypes.c_uint32] * 5 +
                                  [_vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.POINTER(ctypes.c_uint32),
                                   ctypes.POINTER(ctypes.c_double)]),
    "srsgpu_rxq_set_affinity": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32]),
    "srsgpu_rxq_free_host": (_i32, [_vp, _vp]),
    "srsgpu_dlsch_join_tail": (_i32, [_vp]),
    "srsgpu_dlsch_cb_halfits": (_i32, [_vp, _vp, _u32]),
    "srsgpu_rxq_set_input_format": (_i32, [_vp, _u32, ctypes.c_float]),
    "srsgpu_rxq_ingest_stats": (None, [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "srsgpu_rxq_get_chest": (_vp, [_vp]),
    "srsgpu_rxq_get_pdsch": (_vp, [_vp]),
    "srsgpu_rxq_submit_ue_dl": (_i32, [_vp, _vp, ctypes.POINTER(ctypes.c_uint64)]),
    "srsgpu_rxq_decode_rnti": (_i32, [_vp, _vp]),
    "srsgpu_rxq_set_phich": (_i32, [_vp, _u32, _u32]),
    "srsgpu_dlsch_set_early_stop": (None, [_vp, _i32]),
    "srsgpu_dlsch_set_tail_stream": (_i32, [_vp, _vp]),
    "srsgpu_dlsch_set_llr_8bit": (None, [_vp, _i32]),
    "srsgpu_dlsch_set_direct_derm": (None, [_vp, _i32]),
    "srsgpu_rm_turbo_rx_8bit_dev": (_i32, [_vp, _vp, _vp, _u32, _u32, _u32]),
    "srsgpu_pdsch_set_noise_dev": (None, [_vp, _vp]),
    "srsgpu_pdsch_get_dlsch": (_vp, [_vp]),
    "srsgpu_pdsch_llr_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_pdsch_sf_t), _u32, _vp, _vp, _sz, _vp,
                                    ctypes.POINTER(ctypes.c_uint64)]),
    "srsgpu_pdsch_decode_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_pdsch_sf_t), _u32, _vp, _vp, _sz,
                                       _vp, _u32, _vp, _vp]),
    "srsgpu_pdsch_nof_re": (_i32, [ctypes.POINTER(srsgpu_cell_t), ctypes.POINTER(srsgpu_pdsch_sf_t)]),
    "srsgpu_chest_create": (_i32, [ctypes.POINTER(_vp), ctypes.POINTER(srsgpu_cell_t), _u32]),
    "srsgpu_chest_destroy": (None, [_vp]),
    "srsgpu_chest_set_stream": (None, [_vp, _vp]),
    "srsgpu_chest_set_smooth_filter": (_i32, [_vp, ctypes.POINTER(ctypes.c_float), _u32]),
    "srsgpu_chest_set_smooth_filter3_coeff": (None, [_vp, ctypes.c_float]),
    "srsgpu_chest_set_smooth_filter_gauss": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_float]),
    "srsgpu_chest_estimate_dev": (_i32, [_vp, _u32p, _u32, _vp, _sz, _vp, _vp]),
    "srsgpu_pdsch_decode_out_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_pdsch_sf_t), _u32, _vp, _vp, _sz,
                                           ctypes.POINTER(_vp), _u32, _vp, _vp]),
    "srsgpu_dlsch_decode_out_dev": (_i32, [_vp, _vp, _u32, _vp, ctypes.POINTER(_vp), _u32, _vp, _vp]),
    "srsgpu_pdsch_feedback_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_feedback_sf_t), _u32, _vp, _sz, _vp, _vp]),
    "srsgpu_chest_estimate_meas_dev": (_i32, [_vp, _u32p, _u32, _vp, _sz, _vp, _vp, _vp]),
    "srsgpu_chest_set_cfg": (_i32, [_vp, _vp]),
    "srsgpu_chest_get_cfg": (_i32, [_vp, _vp]),
    "srsgpu_symbol_sz": (_i32, [_u32, _i32]),
    "srsgpu_ofdm_rx_create": (_i32, [ctypes.POINTER(_vp), _u32, _u32]),
    "srsgpu_ofdm_rx_destroy": (None, [_vp]),
    "srsgpu_ofdm_rx_set_stream": (None, [_vp, _vp]),
    "srsgpu_ofdm_rx_set_normalize": (None, [_vp, _i32]),
    "srsgpu_ofdm_set_cp": (_i32, [_vp, _u32]),
    "srsgpu_ofdm_rx_sf_dev": (_i32, [_vp, _u32, _vp, _sz, _vp, _sz]),
    "srsgpu_ofdm_tx_sf_dev": (_i32, [_vp, _u32, _vp, _sz, _vp, _sz]),
    "srsgpu_chest_put_crs_dev": (_i32, [_vp, _u32p, _u32, _vp, _sz]),
    "srsgpu_pdsch_encode_ports_dev": (_i32, [_vp, _vp, _u32, _vp, _vp, _sz]),
    "srsgpu_pdsch_encode_dev": (_i32, [_vp, ctypes.POINTER(srsgpu_pdsch_sf_t), _u32, _vp, _vp]),
    "srsgpu_prof_enable": (None, [_i32]),
    "srsgpu_prof_reset": (None, []),
    "srsgpu_prof_get": (_i32, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                               ctypes.POINTER(ctypes.c_uint64)]),
}
for _name, (_res, _args) in _sig.items():
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_sig)


def _i16(a):
    return a.ctypes.data_as(_i16p)


def _u8(a):
    return a.ctypes.data_as(_u8p)


def input_len(impl, sb_layout, K):
    return _lib.srsgpu_tdec_input_len(impl, sb_layout, K)


def autoimp_get_subblocks(K):
    return _lib.srslte_tdec_autoimp_get_subblocks(K)


class Tdec:
    """srslte_tdec_t (one code block at a time, one half-iteration per iteration() call)."""

    def __init__(self, max_long_cb=6144, dec_type=SRSLTE_TDEC_AUTO):
        self.h = srslte_tdec_t()
        r = _lib.srslte_tdec_init_manual(ctypes.byref(self.h), max_long_cb, dec_type)
        if r != SRSLTE_SUCCESS:
            raise RuntimeError("srslte_tdec_init_manual failed (%d)" % r)

    def force_not_sb(self):
        _lib.srslte_tdec_force_not_sb(ctypes.byref(self.h))

    def new_cb(self, K):
        return _lib.srslte_tdec_new_cb(ctypes.byref(self.h), K)

    def iteration(self, inp, out):
        _lib.srslte_tdec_iteration(ctypes.byref(self.h), _i16(inp), _u8(out))

    def run_all(self, inp, out, nof_iterations, K):
        return _lib.srslte_tdec_run_all(ctypes.byref(self.h), _i16(inp), _u8(out), nof_iterations, K)

    def iteration_8bit(self, inp, out):
        _lib.srslte_tdec_iteration_8bit(ctypes.byref(self.h), inp.ctypes.data_as(_i8p), _u8(out))

    def run_all_8bit(self, inp, out, nof_iterations, K):
        return _lib.srslte_tdec_run_all_8bit(ctypes.byref(self.h), inp.ctypes.data_as(_i8p), _u8(out),
                                             nof_iterations, K)

    def get_nof_iterations(self):
        return _lib.srslte_tdec_get_nof_iterations(ctypes.byref(self.h))

    def free(self):
        if self.h.gpu:
            _lib.srslte_tdec_free(ctypes.byref(self.h))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class TdecBatch:
    """srsgpu_tdec_batch_t: batched decoding of code blocks of one size."""

    def __init__(self, max_cbs, max_long_cb=6144, stream=None):
        self.q = _vp()
        r = _lib.srsgpu_tdec_batch_create(ctypes.byref(self.q), max_cbs, max_long_cb)
        if r != 0:
            raise RuntimeError("srsgpu_tdec_batch_create failed")
        if stream is not None:
            self.set_stream(stream)

    def set_stream(self, stream):
        _lib.srsgpu_tdec_batch_set_stream(self.q, _vp(stream))

    # ---- device pointers (ints) ----
    def run_dev(self, impl, sb, d_in, in_stride, K, n, nhalf, d_out, out_stride):
        return _lib.srsgpu_tdec_batch_run_dev(self.q, impl, sb, _vp(d_in), in_stride, K, n, nhalf,
                                              _vp(d_out), out_stride)

    def decode_dev(self, impl, sb, d_in, in_stride, K, n, maxh, poly, crc_len, d_out, out_stride,
                   d_ok=None, d_noi=None):
        return _lib.srsgpu_tdec_batch_decode_dev(self.q, impl, sb, _vp(d_in), in_stride, K, n,
                                                 maxh, poly, crc_len, _vp(d_out), out_stride,
                                                 _vp(d_ok), _vp(d_noi))

    def read_state(self, cb, K):
        """(app1, ext1) of code block cb after the last half-iteration, reference index space"""
        app1, ext1 = np.zeros(K, np.int16), np.zeros(K, np.int16)
        if _lib.srsgpu_tdec_batch_read_state(self.q, cb, _i16(app1), _i16(ext1)) != 0:
            raise RuntimeError("srsgpu_tdec_batch_read_state failed")
        return app1, ext1

    # ---- host numpy arrays ----
    def run(self, impl, sb, inputs, K, nhalf):
        n = len(inputs)
        ins = [np.ascontiguousarray(x, np.int16) for x in inputs]
        outs = [np.zeros(K // 8, np.uint8) for _ in range(n)]
        ip = (_vp * n)(*[x.ctypes.data for x in ins])
        op = (_vp * n)(*[x.ctypes.data for x in outs])
        r = _lib.srsgpu_tdec_batch_run(self.q, impl, sb, ip, K, n, nhalf, op)
        if r != 0:
            raise RuntimeError("srsgpu_tdec_batch_run failed")
        return np.stack(outs)

    def decode(self, impl, sb, inputs, K, maxh, poly, crc_len):
        n = len(inputs)
        ins = [np.ascontiguousarray(x, np.int16) for x in inputs]
        outs = [np.zeros(K // 8, np.uint8) for _ in range(n)]
        ok = np.zeros(n, np.uint8)
        noi = np.zeros(n, np.uint32)
        ip = (_vp * n)(*[x.ctypes.data for x in ins])
        op = (_vp * n)(*[x.ctypes.data for x in outs])
        r = _lib.srsgpu_tdec_batch_decode(self.q, impl, sb, ip, K, n, maxh, poly, crc_len, op,
                                          ok.ctypes.data_as(_u8p), noi.ctypes.data_as(_u32p))
        if r != 0:
            raise RuntimeError("srsgpu_tdec_batch_decode failed")
        return np.stack(outs), ok, noi

    def close(self):
        if self.q:
            _lib.srsgpu_tdec_batch_destroy(self.q)
            self.q = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Tcod:
    """srslte_tcod_t bit encoder (host): bits in, [s,p0,p1]*K + 12 tail bits out."""

    def __init__(self, max_long_cb=6144):
        self.h = srslte_tcod_t()
        if _lib.srslte_tcod_init(ctypes.byref(self.h), max_long_cb) != 0:
            raise RuntimeError("srslte_tcod_init failed")

    def encode(self, bits):
        bits = np.ascontiguousarray(bits, np.uint8)
        out = np.zeros(3 * bits.size + 12, np.uint8)
        if _lib.srslte_tcod_encode(ctypes.byref(self.h), _u8(bits), _u8(out), bits.size) != 0:
            raise RuntimeError("srslte_tcod_encode failed")
        return out

    def __del__(self):
        try:
            _lib.srslte_tcod_free(ctypes.byref(self.h))
        except Exception:
            pass


class Dlsch:
    """srsgpu_dlsch_t: batched transport-block decoding (de-RM + HARQ, turbo decoding with CRC
    early stop, TB CRC) with device-resident softbuffers."""

    def __init__(self, nof_softbuffers, max_cb=13, max_cbs_per_call=1024, stream=None):
        self.q = _vp()
        self.max_cb = max_cb
        if _lib.srsgpu_dlsch_create(ctypes.byref(self.q), nof_softbuffers, max_cb,
                                    max_cbs_per_call) != 0:
            raise RuntimeError("srsgpu_dlsch_create failed")
        if stream is not None:
            _lib.srsgpu_dlsch_set_stream(self.q, _vp(stream))

    @staticmethod
    def _tbs(tbs_list):
        if isinstance(tbs_list, ctypes.Array):  # prebuilt descriptors (make_tb_array)
            return tbs_list
        arr = (srsgpu_dlsch_tb_t * len(tbs_list))()
        for i, t in enumerate(tbs_list):
            for k, v in t.items():
                setattr(arr[i], k, v)
        return arr

    def reset(self, slot, tbs=None):
        r = (_lib.srsgpu_dlsch_softbuffer_reset(self.q, slot) if tbs is None
             else _lib.srsgpu_dlsch_softbuffer_reset_tbs(self.q, slot, tbs))
        if r != 0:
            raise RuntimeError("softbuffer reset failed")

    def set_early_stop(self, on):
        """srsgpu_dlsch_set_early_stop (off: every CB runs max_halfits, one CRC check at the end)"""
        _lib.srsgpu_dlsch_set_early_stop(self.q, int(bool(on)))

    def set_tail_stream(self, stream):
        """srsgpu_dlsch_set_tail_stream: the early-stop tail of each decode call on `stream` (a HIP
        stream handle, 0 = off)"""
        if _lib.srsgpu_dlsch_set_tail_stream(self.q, _vp(stream or None)) != 0:
            raise RuntimeError("srsgpu_dlsch_set_tail_stream failed")

    def join_tail(self):
        """srsgpu_dlsch_join_tail: the engine's stream waits for its last call's tail (tail stream)"""
        if _lib.srsgpu_dlsch_join_tail(self.q) != 0:
            raise RuntimeError("srsgpu_dlsch_join_tail failed")

    def set_direct_derm(self, on):
        """srsgpu_dlsch_set_direct_derm (off: every softbuffer row written before the decode)"""
        _lib.srsgpu_dlsch_set_direct_derm(self.q, int(bool(on)))

    def reset_range(self, first, count):
        if _lib.srsgpu_dlsch_softbuffer_reset_range(self.q, first, count) != 0:
            raise RuntimeError("softbuffer reset failed")

    def decode(self, tbs_list, e_bits, max_halfits=8):
        """tbs_list: dicts {tbs, rv, Qm, nof_e_bits, softbuffer}; e_bits: int16 arrays.
        Returns (ret[], data[], noi[])."""
        n = len(tbs_list)
        arr = self._tbs(tbs_list)
        es = [np.ascontiguousarray(e, np.int16) for e in e_bits]
        outs = [np.zeros(dlsch_data_len(t["tbs"]), np.uint8) for t in tbs_list]
        ep = (_vp * n)(*[e.ctypes.data for e in es])
        op = (_vp * n)(*[o.ctypes.data for o in outs])
        ret = (ctypes.c_int32 * n)()
        noi = np.zeros(n, np.uint32)
        if _lib.srsgpu_dlsch_decode(self.q, arr, n, ep, op, max_halfits, ret,
                                    noi.ctypes.data_as(_u32p)) != 0:
            raise RuntimeError("srsgpu_dlsch_decode failed")
        return list(ret), outs, noi

    def decode_dev(self, tbs_list, d_e, d_data, max_halfits, d_ret, d_noi):
        arr = self._tbs(tbs_list)
        return _lib.srsgpu_dlsch_decode_dev(self.q, arr, len(tbs_list), _vp(d_e), _vp(d_data),
                                            max_halfits, _vp(d_ret), _vp(d_noi))

    def ulsch_decode_dev(self, tbs_list, d_q, d_g, d_data, max_halfits, d_ret, d_noi):
        """srsgpu_ulsch_decode_dev (srslte_ulsch_decode): tbs_list of dicts with tbs, rv, Qm,
        nof_bits, nof_symb, softbuffer, q_offset, data_offset"""
        arr = (srsgpu_ulsch_tb_t * len(tbs_list))(*[
            srsgpu_ulsch_tb_t(t["tbs"], t["rv"], t["Qm"], t["nof_bits"], t["nof_symb"], t["softbuffer"],
                              t["q_offset"], t["data_offset"]) for t in tbs_list])
        return _lib.srsgpu_ulsch_decode_dev(self.q, arr, len(tbs_list), _vp(d_q), _vp(d_g), _vp(d_data),
                                            max_halfits, _vp(d_ret), _vp(d_noi))

    def ulsch_uci_decode_dev(self, tbs_list, uci_list, d_q, d_c, d_g, d_data, max_halfits, d_ret, d_noi, d_uci):
        """srsgpu_ulsch_uci_decode_dev (srslte_pusch_decode's UCI and data steps): tbs_list as for
        ulsch_decode_dev, uci_list of dicts O (ack, ri, cqi), I_off (ack, ri, cqi), M_sc, M_sc_init,
        c_offset; d_q scrambled soft bits, d_c scrambling bytes, d_uci srsgpu_uci_result_t[n]"""
        n = len(tbs_list)
        arr = (srsgpu_ulsch_tb_t * n)(*[
            srsgpu_ulsch_tb_t(t["tbs"], t["rv"], t["Qm"], t["nof_bits"], t["nof_symb"], t["softbuffer"],
                              t["q_offset"], t["data_offset"]) for t in tbs_list])
        ua = (srsgpu_uci_cfg_t * n)(*[
            srsgpu_uci_cfg_t(u["O"][0], u["O"][1], u["O"][2], u["I_off"][0], u["I_off"][1], u["I_off"][2], u["M_sc"],
                             u["M_sc_init"], u["c_offset"]) for u in uci_list])
        return _lib.srsgpu_ulsch_uci_decode_dev(self.q, arr, ua, n, _vp(d_q), _vp(d_c), _vp(d_g), _vp(d_data),
                                                max_halfits, _vp(d_ret), _vp(d_noi), _vp(d_uci))

    def read_cb_crc(self, slot):
        """cb_crc flags of softbuffer `slot` (the soft bits are not copied)"""
        crc = np.zeros(self.max_cb, np.uint8)
        if _lib.srsgpu_dlsch_softbuffer_read(self.q, slot, None, _u8(crc)) != 0:
            raise RuntimeError("softbuffer read failed")
        return crc

    def cb_halfits(self, max_cbs=1 << 16):
        """srsgpu_dlsch_cb_halfits: the half-iterations of every code block of the last decode call"""
        out = np.zeros(max_cbs, np.uint32)
        n = _lib.srsgpu_dlsch_cb_halfits(self.q, out.ctypes.data, max_cbs)
        if n < 0:
            raise RuntimeError("srsgpu_dlsch_cb_halfits failed")
        return out[:min(n, max_cbs)]

    def read_softbuffer(self, slot):
        rows = np.zeros((self.max_cb, SOFTBUFFER_SIZE), np.int16)
        crc = np.zeros(self.max_cb, np.uint8)
        if _lib.srsgpu_dlsch_softbuffer_read(self.q, slot, _i16(rows), _u8(crc)) != 0:
            raise RuntimeError("softbuffer read failed")
        return rows, crc

    def encode_dev(self, tbs_list, d_data, d_e):
        """srsgpu_dlsch_encode_dev: tbs_list as for decode (dicts with tbs, rv, Qm, nof_e_bits,
        e_offset, data_offset)"""
        arr = self._tbs(tbs_list)
        return _lib.srsgpu_dlsch_encode_dev(self.q, arr, len(tbs_list), _vp(d_data), _vp(d_e))

    def rm_rx_dev(self, d_in, d_out, in_len, K, rv, sb_layout):
        return _lib.srsgpu_rm_turbo_rx_dev(self.q, _vp(d_in), _vp(d_out), in_len, K, rv, sb_layout)

    def set_llr_8bit(self, on):
        """srslte_sch_t.llr_is_8bit: e_bits hold int8 values (int16 elements)"""
        _lib.srsgpu_dlsch_set_llr_8bit(self.q, 1 if on else 0)

    def rm_rx_8bit_dev(self, d_in, d_out, in_len, K, rv):
        return _lib.srsgpu_rm_turbo_rx_8bit_dev(self.q, _vp(d_in), _vp(d_out), in_len, K, rv)

    def close(self):
        if self.q:
            _lib.srsgpu_dlsch_destroy(self.q)
            self.q = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_sf(sf_idx=1, lstart=1, prb=None, nof_prb=100, mod=3, nof_re=0, rnti=1234, noise=0.0,
            scaling=1.0, tbs=0, rv=0, softbuffer=0, grid_offset=0, data_offset=0, mimo=0,
            ce_offset=None, tb_cw_swap=0, codebook_idx=0):
    """srsgpu_pdsch_sf_t from keyword arguments; prb: None (all) or a (2, nof_prb) 0/1 array.
    Per-TB fields (mod, tbs, rv, softbuffer, data_offset) take a value or a (tb0, tb1) pair;
    ce_offset defaults to grid_offset (1-port cells: one estimate plane per rx antenna)."""
    s = srsgpu_pdsch_sf_t()
    s.sf_idx, s.lstart, s.nof_re, s.rnti = sf_idx, lstart, nof_re, rnti
    s.noise_estimate, s.scaling, s.mimo_type, s.tb_cw_swap = noise, scaling, mimo, tb_cw_swap
    s.codebook_idx = codebook_idx
    for name, v in (("mod", mod), ("tbs", tbs), ("rv", rv), ("softbuffer", softbuffer),
                    ("data_offset", data_offset)):
        pair = tuple(v) if isinstance(v, (tuple, list)) else (v, 0)
        getattr(s, name)[0], getattr(s, name)[1] = pair
    s.grid_offset = grid_offset
    s.ce_offset = grid_offset if ce_offset is None else ce_offset
    m = np.ones((2, nof_prb), np.uint8) if prb is None else np.asarray(prb, np.uint8)
    for sl in range(2):
        for n in range(m.shape[1]):
            s.prb_idx[sl][n] = int(m[sl, n])
    return s


def make_tb_array(tbs_list):
    """srsgpu_dlsch_tb_t[] from dicts, built once and reusable across calls"""
    return Dlsch._tbs(tbs_list)


def make_sf_array(sfs):
    """srsgpu_pdsch_sf_t[] from make_sf() results, built once and reusable across calls"""
    return sfs if isinstance(sfs, ctypes.Array) else (srsgpu_pdsch_sf_t * len(sfs))(*sfs)


class Pcfich:
    """srsgpu_pcfich_t: batched srslte_pcfich_decode_multi (CFI detection) on device grids laid
    out as Pdsch's (include/srsgpu/pcfich_batch.h)."""

    def __init__(self, nof_prb, cell_id, nof_ports=1, nof_rx_ant=1, cp=0):
        self.cell = srsgpu_cell_t(nof_prb, cell_id, nof_ports, nof_rx_ant, cp)
        self.q = _vp()
        if _lib.srsgpu_pcfich_create(ctypes.byref(self.q), ctypes.byref(self.cell)) != 0:
            raise RuntimeError("srsgpu_pcfich_create failed")

    def re_map(self):
        idx = (ctypes.c_uint32 * 16)()
        assert _lib.srsgpu_pcfich_re_map(self.q, idx) == 16
        return list(idx)

    @staticmethod
    def make_sf_array(sfs):
        """list of (grid_offset, ce_offset, sf_idx, noise_estimate) -> srsgpu_pcfich_sf_t array"""
        arr = (srsgpu_pcfich_sf_t * max(len(sfs), 1))()
        for i, (g, c, sf, n) in enumerate(sfs):
            arr[i].grid_offset, arr[i].ce_offset, arr[i].sf_idx, arr[i].noise_estimate = g, c, sf, n
        return arr

    def decode_dev(self, sfs, d_grid, d_ce, ant_stride, d_cfi, d_corr, stream=None):
        """sfs: list of (grid_offset, ce_offset, sf_idx, noise_estimate), or (array, count) from
        make_sf_array"""
        arr, n = sfs if isinstance(sfs, tuple) else (self.make_sf_array(sfs), len(sfs))
        return _lib.srsgpu_pcfich_decode_dev(self.q, arr, n, _vp(d_grid), _vp(d_ce), ant_stride,
                                             _vp(d_cfi), _vp(d_corr), _vp(stream))

    def __del__(self):
        if getattr(self, "q", None):
            _lib.srsgpu_pcfich_destroy(self.q)
            self.q = None


def pdcch_cell_map(nof_prb, cell_id, nof_ports, phich_length, phich_resources, cfi, cp=0):
    """srsgpu_pdcch_cell_map (host only): (grid indices of the PDCCH symbols in srslte_regs_pdcch_get
    order, NOF_CCE(cfi)); None for an invalid cell"""
    cell = srsgpu_cell_t(nof_prb, cell_id, nof_ports, 1, cp)
    ncce = ctypes.c_uint32(0)
    n = _lib.srsgpu_pdcch_cell_map(ctypes.byref(cell), phich_length, phich_resources, cfi, None, 0,
                                   ctypes.byref(ncce))
    if n < 0:
        return None
    idx = np.zeros(max(n, 1), np.uint32)
    assert _lib.srsgpu_pdcch_cell_map(ctypes.byref(cell), phich_length, phich_resources, cfi,
                                      idx.ctypes.data_as(_u32p), n, None) == n
    return idx[:n], ncce.value


def pdcch_locations(nof_cce, sf_idx=0, rnti=0, common=False):
    """srsgpu_pdcch_ue_locations / _common_locations: [(L, ncce)] in the reference's order"""
    c = (srsgpu_dci_location_t * 64)()
    n = (_lib.srsgpu_pdcch_common_locations(nof_cce, c, 64) if common
         else _lib.srsgpu_pdcch_ue_locations(nof_cce, sf_idx, rnti, c, 64))
    return [(c[i].L, c[i].ncce) for i in range(n)]


def dci_format_sizeof(fmt, nof_prb, nof_ports):
    return _lib.srsgpu_dci_format_sizeof(fmt, nof_prb, nof_ports)


def dci_msg_to_ul_grant(bits, nof_prb, n_rb_ho=0, nof_bits=None):
    """srsgpu_dci_msg_to_ul_grant -> (ret, srsgpu_ra_ul_dci_t, srsgpu_ra_ul_grant_t)"""
    b = np.zeros(128, np.uint8)
    b[:len(bits)] = bits
    nof_bits = len(bits) if nof_bits is None else nof_bits
    d, g = srsgpu_ra_ul_dci_t(), srsgpu_ra_ul_grant_t()
    r = _lib.srsgpu_dci_msg_to_ul_grant(b.ctypes.data_as(_u8p), nof_bits, nof_prb, n_rb_ho, ctypes.byref(d),
                                        ctypes.byref(g))
    return r, d, g


def dci_msg_to_dl_grant(bits, fmt, rnti, nof_prb, nof_ports, nof_bits=None):
    """srsgpu_dci_msg_to_dl_grant of bits[:nof_bits] (default: all of bits), read from a zero-padded
    128-byte message buffer: (ret, srsgpu_ra_dl_dci_t, srsgpu_ra_dl_grant_t)"""
    b = np.zeros(128, np.uint8)
    b[:len(bits)] = bits
    nof_bits = len(bits) if nof_bits is None else nof_bits
    d, g = srsgpu_ra_dl_dci_t(), srsgpu_ra_dl_grant_t()
    r = _lib.srsgpu_dci_msg_to_dl_grant(b.ctypes.data_as(_u8p), nof_bits, fmt, rnti, nof_prb, nof_ports,
                                        ctypes.byref(d), ctypes.byref(g))
    return r, d, g


class Pdcch:
    """srsgpu_pdcch_t: batched srslte_pdcch_extract_llr_multi and the srslte_ue_dl_find_dl_dci blind
    search on device grids laid out as Pdsch's (include/srsgpu/pdcch_batch.h)."""

    def __init__(self, nof_prb, cell_id, nof_ports=1, nof_rx_ant=1, phich_length=0, phich_resources=0, cp=0):
        self.cell = srsgpu_cell_t(nof_prb, cell_id, nof_ports, nof_rx_ant, cp)
        self.q = _vp()
        if _lib.srsgpu_pdcch_create(ctypes.byref(self.q), ctypes.byref(self.cell), phich_length,
                                    phich_resources) != 0:
            raise RuntimeError("srsgpu_pdcch_create failed")

    def nof_cce(self, cfi):
        return _lib.srsgpu_pdcch_nof_cce(self.q, cfi)

    def re_map(self, cfi):
        idx = np.zeros(36 * max(self.nof_cce(cfi), 1), np.uint32)
        n = _lib.srsgpu_pdcch_re_map(self.q, cfi, idx.ctypes.data_as(_u32p), idx.size)
        assert n >= 0
        return idx[:n]

    @staticmethod
    def make_sf_array(sfs):
        """list of (grid_offset, ce_offset, llr_offset, sf_idx, cfi, noise) -> srsgpu_pdcch_sf_t array"""
        arr = (srsgpu_pdcch_sf_t * max(len(sfs), 1))()
        for i, (g, c, l, sf, cfi, n) in enumerate(sfs):
            arr[i].grid_offset, arr[i].ce_offset, arr[i].llr_offset = g, c, l
            arr[i].sf_idx, arr[i].cfi, arr[i].noise_estimate = sf, cfi, n
        return arr

    def extract_llr_dev(self, sfs, d_grid, d_ce, ant_stride, d_llr, stream=None):
        arr, n = sfs if isinstance(sfs, tuple) else (self.make_sf_array(sfs), len(sfs))
        return _lib.srsgpu_pdcch_extract_llr_dev(self.q, arr, n, _vp(d_grid), _vp(d_ce), ant_stride,
                                                 _vp(d_llr), _vp(stream))

    @staticmethod
    def make_search_array(searches):
        """list of (llr_offset, sf_idx, cfi, rnti, tm[, rnti_type[, ul_rnti]]) -> srsgpu_dci_search_t array"""
        arr = (srsgpu_dci_search_t * max(len(searches), 1))()
        for i, s in enumerate(searches):
            arr[i].llr_offset, arr[i].sf_idx, arr[i].cfi, arr[i].rnti, arr[i].tm = s[:5]
            arr[i].rnti_type = s[5] if len(s) > 5 else -1
            arr[i].ul_rnti = s[6] if len(s) > 6 else 0
        return arr

    def find_dci_dev(self, searches, d_llr, d_res, d_res_ul, stream=None):
        """srsgpu_pdcch_find_dci_dev: DL then UL searches; d_res / d_res_ul: len(searches) results each"""
        arr = self.make_search_array(searches)
        return _lib.srsgpu_pdcch_find_dci_dev(self.q, arr, len(searches), _vp(d_llr), _vp(d_res), _vp(d_res_ul),
                                              _vp(stream))

    def find_dl_dci_dev(self, searches, d_llr, d_res, stream=None):
        """d_res: device buffer of len(searches) srsgpu_dci_result_t (RESULT_SIZE bytes each)"""
        arr = self.make_search_array(searches)
        return _lib.srsgpu_pdcch_find_dl_dci_dev(self.q, arr, len(searches), _vp(d_llr), _vp(d_res),
                                                 _vp(stream))

    RESULT_SIZE = ctypes.sizeof(srsgpu_dci_result_t)

    @staticmethod
    def parse_results(raw):
        """bytes of n srsgpu_dci_result_t -> [(found 1 / 0 / -1, format, L, ncce, the 128-byte message
        buffer)]"""
        raw = bytes(raw)
        n = len(raw) // ctypes.sizeof(srsgpu_dci_result_t)
        out = []
        for i in range(n):
            r = srsgpu_dci_result_t.from_buffer_copy(raw, i * ctypes.sizeof(srsgpu_dci_result_t))
            out.append((r.found, r.format, r.L, r.ncce, np.array(r.data[:], np.uint8) if r.found > 0
                        else np.zeros(0, np.uint8)))
        return out

    def __del__(self):
        if getattr(self, "q", None):
            _lib.srsgpu_pdcch_destroy(self.q)
            self.q = None


class Pdsch:
    """srsgpu_pdsch_t: batched PDSCH receive (RE extraction, SISO equalisation, demapping,
    descrambling, CSI, DL-SCH decoding) on device grids."""

    def __init__(self, nof_prb, cell_id, nof_ports=1, nof_rx_ant=1, nof_softbuffers=16, max_cb=13,
                 max_sf=64, stream=None, cp=0):
        self.cell = srsgpu_cell_t(nof_prb, cell_id, nof_ports, nof_rx_ant, cp)
        self.q = _vp()
        if _lib.srsgpu_pdsch_create(ctypes.byref(self.q), ctypes.byref(self.cell), nof_softbuffers,
                                    max_cb, max_sf) != 0:
            raise RuntimeError("srsgpu_pdsch_create failed")
        if stream is not None:
            _lib.srsgpu_pdsch_set_stream(self.q, _vp(stream))
        self.dlsch_q = _lib.srsgpu_pdsch_get_dlsch(self.q)

    def set_csi(self, on):
        _lib.srsgpu_pdsch_set_csi(self.q, 1 if on else 0)

    def set_ce_rows(self, rows):
        """srsgpu_pdsch_set_ce_rows: 0 full estimate planes, 4 / 1 the chest's compact rows"""
        if _lib.srsgpu_pdsch_set_ce_rows(self.q, rows) != 0:
            raise ValueError("invalid ce_rows")

    def set_llr_8bit(self, on):
        """srslte_pdsch_t.llr_is_8bit: int8 LLR chain (values held in the int16 LLR elements)"""
        _lib.srsgpu_pdsch_set_llr_8bit(self.q, 1 if on else 0)

    def set_noise_dev(self, d_noise):
        _lib.srsgpu_pdsch_set_noise_dev(self.q, _vp(d_noise) if d_noise else None)

    def reset_softbuffer(self, slot, count=None):
        r = (_lib.srsgpu_dlsch_softbuffer_reset(_vp(self.dlsch_q), slot) if count is None else
             _lib.srsgpu_dlsch_softbuffer_reset_range(_vp(self.dlsch_q), slot, count))
        if r != 0:
            raise RuntimeError("softbuffer reset failed")

    def nof_re(self, sf):
        return _lib.srsgpu_pdsch_nof_re(ctypes.byref(self.cell), ctypes.byref(sf))

    def read_cb_crc(self, slot, max_cb=13):
        """cb_crc flags of softbuffer `slot` of the PDSCH's DL-SCH (srsgpu_dlsch_softbuffer_read)"""
        crc = np.zeros(max_cb, np.uint8)
        if _lib.srsgpu_dlsch_softbuffer_read(_vp(self.dlsch_q), slot, None, _u8(crc)) != 0:
            raise RuntimeError("softbuffer read failed")
        return crc

    def llr_dev(self, sfs, d_grid, d_ce, ant_stride, d_e, e_offsets):
        arr = make_sf_array(sfs)
        offs = e_offsets if isinstance(e_offsets, ctypes.Array) else \
            (ctypes.c_uint64 * len(e_offsets))(*e_offsets)  # one per TB
        return _lib.srsgpu_pdsch_llr_dev(self.q, arr, len(sfs), _vp(d_grid), _vp(d_ce), ant_stride,
                                         _vp(d_e), offs)

    def encode_dev(self, sfs, d_data, d_grid, port_stride=None):
        """srsgpu_pdsch_encode_dev: TB bytes (data_offset[0]) -> PDSCH REs of each grid; with port_stride
        srsgpu_pdsch_encode_ports_dev (every MIMO type, port p's grid port_stride elements after p - 1)"""
        arr, n = (sfs if isinstance(sfs, tuple) else (make_sf_array(sfs), len(sfs)))
        if port_stride is None:
            return _lib.srsgpu_pdsch_encode_dev(self.q, arr, n, _vp(d_data), _vp(d_grid))
        return _lib.srsgpu_pdsch_encode_ports_dev(self.q, arr, n, _vp(d_data), _vp(d_grid), port_stride)

    def decode_dev(self, sfs, d_grid, d_ce, ant_stride, d_data, max_halfits, d_ret, d_noi):
        arr = make_sf_array(sfs)
        return _lib.srsgpu_pdsch_decode_dev(self.q, arr, len(sfs), _vp(d_grid), _vp(d_ce), ant_stride,
                                            _vp(d_data), max_halfits, _vp(d_ret), _vp(d_noi))

    def feedback_dev(self, items, d_ce, ant_stride, d_out, d_noise=None):
        """srsgpu_pdsch_feedback_dev: items of (ce_offset, noise_estimate, flags); d_out device memory of
        len(items) srsgpu_feedback_t"""
        arr = (srsgpu_feedback_sf_t * len(items))(*[srsgpu_feedback_sf_t(o, nz, f) for o, nz, f in items])
        return _lib.srsgpu_pdsch_feedback_dev(self.q, arr, len(items), _vp(d_ce), ant_stride, _vp(d_noise), _vp(d_out))

    @staticmethod
    def parse_feedback(raw, n):
        return list((srsgpu_feedback_t * n).from_buffer_copy(raw[:n * ctypes.sizeof(srsgpu_feedback_t)]))

    def close(self):
        if self.q:
            _lib.srsgpu_pdsch_destroy(self.q)
            self.q = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class srsgpu_chest_cfg_t(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("average_subframe", "noise_alg", "smooth_filter_auto",
                                               "rsrp_neighbour", "cfo_estimate_enable",
                                               "cfo_estimate_sf_mask", "symbol_sz")]


class Chest:
    """srsgpu_chest_t: batched CRS channel estimation (ports 0/1, normal CP) on device grids.
    With nof_ports = 2 grid i yields estimates i*2 (port 0) and i*2 + 1 (port 1)."""

    def __init__(self, nof_prb, cell_id, max_grids=64, stream=None, nof_ports=1, cp=0):
        self.cell = srsgpu_cell_t(nof_prb, cell_id, nof_ports, 1, cp)
        self.q = _vp()
        if _lib.srsgpu_chest_create(ctypes.byref(self.q), ctypes.byref(self.cell), max_grids) != 0:
            raise RuntimeError("srsgpu_chest_create failed")
        if stream is not None:
            _lib.srsgpu_chest_set_stream(self.q, _vp(stream))

    def set_filter(self, taps):
        arr = (ctypes.c_float * max(1, len(taps)))(*taps)
        if _lib.srsgpu_chest_set_smooth_filter(self.q, arr, len(taps)) != 0:
            raise RuntimeError("invalid smoothing filter")

    def set_filter3(self, w):
        _lib.srsgpu_chest_set_smooth_filter3_coeff(self.q, w)

    def set_ce_rows(self, on):
        """srsgpu_chest_set_ce_rows: compact estimate rows (4, or 1 with average_subframe)"""
        _lib.srsgpu_chest_set_ce_rows(self.q, int(bool(on)))

    def set_filter_gauss(self, order, std_dev):
        if _lib.srsgpu_chest_set_smooth_filter_gauss(self.q, order, ctypes.c_float(std_dev)) != 0:
            raise RuntimeError("invalid Gaussian smoothing filter")

    def put_crs_dev(self, sf_idx, d_grid, stride):
        n = len(sf_idx)
        arr = sf_idx if isinstance(sf_idx, ctypes.Array) else (ctypes.c_uint32 * n)(*sf_idx)
        return _lib.srsgpu_chest_put_crs_dev(self.q, arr, n, _vp(d_grid), stride)

    def set_cfg(self, average_subframe=False, noise_alg=0, smooth_filter_auto=False,
                rsrp_neighbour=False, cfo_enable=False, cfo_mask=0, symbol_sz=None):
        """srsgpu_chest_cfg_t; noise_alg 0 REFS, 1 PSS, 2 EMPTY"""
        c = srsgpu_chest_cfg_t(int(average_subframe), noise_alg, int(smooth_filter_auto), int(rsrp_neighbour),
                               int(cfo_enable), cfo_mask, symbol_sz or symbol_sz_of(self.cell.nof_prb))
        if _lib.srsgpu_chest_set_cfg(self.q, ctypes.byref(c)) != 0:
            raise RuntimeError("invalid chest configuration")

    def estimate_meas_dev(self, sf_idx, d_grid, stride, d_ce, d_noise=None, d_meas=None):
        n = len(sf_idx)
        arr = sf_idx if isinstance(sf_idx, ctypes.Array) else (ctypes.c_uint32 * n)(*sf_idx)
        return _lib.srsgpu_chest_estimate_meas_dev(self.q, arr, n, _vp(d_grid), stride, _vp(d_ce),
                                                   _vp(d_noise) if d_noise else None,
                                                   _vp(d_meas) if d_meas else None)

    def estimate_dev(self, sf_idx, d_grid, stride, d_ce, d_noise=None):
        n = len(sf_idx)
        arr = sf_idx if isinstance(sf_idx, ctypes.Array) else (ctypes.c_uint32 * n)(*sf_idx)
        return _lib.srsgpu_chest_estimate_dev(self.q, arr, n, _vp(d_grid), stride, _vp(d_ce),
                                              _vp(d_noise) if d_noise else None)

    def close(self):
        if self.q:
            _lib.srsgpu_chest_destroy(self.q)
            self.q = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def symbol_sz_of(nof_prb):
    """srslte_symbol_sz without standard rates (phy_common.c:245-264)"""
    return next(sz for lim, sz in ((6, 128), (15, 256), (25, 384), (50, 768), (75, 1024), (110, 1536))
                if nof_prb <= lim)


def symbol_sz(nof_prb, standard_rates=False):
    return _lib.srsgpu_symbol_sz(nof_prb, 1 if standard_rates else 0)


class OfdmRx:
    """srsgpu_ofdm_t: batched OFDM receive FFT (normal CP, or extended with cp=1) on device sample
    buffers."""

    def __init__(self, nof_prb, symbol_size, normalize=False, stream=None, cp=0):
        self.q = _vp()
        if _lib.srsgpu_ofdm_rx_create(ctypes.byref(self.q), nof_prb, symbol_size) != 0:
            raise RuntimeError("srsgpu_ofdm_rx_create failed")
        _lib.srsgpu_ofdm_rx_set_normalize(self.q, 1 if normalize else 0)
        if _lib.srsgpu_ofdm_set_cp(self.q, cp) != 0:
            raise RuntimeError("srsgpu_ofdm_set_cp failed")
        if stream is not None:
            _lib.srsgpu_ofdm_rx_set_stream(self.q, _vp(stream))

    def rx_dev(self, n, d_in, in_stride, d_out, out_stride):
        return _lib.srsgpu_ofdm_rx_sf_dev(self.q, n, _vp(d_in), in_stride, _vp(d_out), out_stride)

    def tx_dev(self, n, d_in, in_stride, d_out, out_stride):
        """srsgpu_ofdm_tx_sf_dev: grids -> time-domain subframes (same handle)"""
        return _lib.srsgpu_ofdm_tx_sf_dev(self.q, n, _vp(d_in), in_stride, _vp(d_out), out_stride)

    def close(self):
        if self.q:
            _lib.srsgpu_ofdm_rx_destroy(self.q)
            self.q = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def prof_enable(on=True):
    _lib.srsgpu_prof_enable(1 if on else 0)


def prof_reset():
    _lib.srsgpu_prof_reset()


def prof_get(name):
    t = ctypes.c_double(0)
    c = ctypes.c_uint64(0)
    _lib.srsgpu_prof_get(name.encode() if name else None, ctypes.byref(t), ctypes.byref(c))
    return t.value, c.value


def shard_contiguous(n, world):
    """srsgpu_shard_contiguous: rank r owns units [first[r], first[r + 1])"""
    first = (ctypes.c_uint32 * (world + 1))()
    if _lib.srsgpu_shard_contiguous(n, world, first) != 0:
        raise ValueError("invalid partition request (n=%d, world=%d)" % (n, world))
    return list(first)


def shard_weighted(weights, world):
    """srsgpu_shard_weighted: (owner per unit, summed weight per rank), global LPT queue"""
    w = np.ascontiguousarray(weights, np.uint64)
    owner = np.zeros(w.size, np.int32)
    load = np.zeros(world, np.uint64)
    if _lib.srsgpu_shard_weighted(w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), w.size, world,
                                  owner.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                  load.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))) != 0:
        raise ValueError("invalid partition request (n=%d, world=%d)" % (w.size, world))
    return owner, load


def set_schedule(fused=-1, es_fused=-1, es_chunk=-1, sse_bidir=-1):
    """srsgpu_tdec_set_schedule: the decoder launch schedule (results are identical under all)"""
    if _lib.srsgpu_tdec_set_schedule(fused, es_fused, es_chunk, sse_bidir) != 0:
        raise ValueError("invalid decoder schedule")


def knobs_reload():
    """srsgpu_knobs_reload: re-read the launch knobs (SRSGPU_*_PRIO, SRSGPU_LLR_*) after os.environ
    changed them; the library reads them once otherwise"""
    _lib.srsgpu_knobs_reload()


def get_schedule():
    v = [ctypes.c_int(0) for _ in range(4)]
    _lib.srsgpu_tdec_get_schedule(*[ctypes.byref(x) for x in v])
    return dict(zip(("fused", "es_fused", "es_chunk", "sse_bidir"), (x.value for x in v)))


class RxQueue:
    """srsgpu_rxq_t (include/srsgpu/rx_queue.h): PHY-worker threads hand over single time-domain
    subframes; one dispatcher thread decodes them in batches (OFDM -> chest -> PDSCH / DL-SCH)."""

    def __init__(self, nof_prb, cell_id, symbol_sz, nof_ports=1, nof_rx_ant=1, nof_softbuffers=16,
                 max_batch=32, max_wait_us=500, max_halfits=8, cp=0):
        self.cell = srsgpu_cell_t(nof_prb, cell_id, nof_ports, nof_rx_ant, cp)
        self.q = _vp()
        if _lib.srsgpu_rxq_create(ctypes.byref(self.q), ctypes.byref(self.cell), symbol_sz,
                                  nof_softbuffers, max_batch, max_wait_us, max_halfits) != 0:
            raise RuntimeError("srsgpu_rxq_create failed")

    @staticmethod
    def item(td, sf, data, reset=(1, 0)):
        """td: complex64 arrays per rx antenna (kept alive by the caller); data: uint8 output arrays
        per TB; sf: make_sf(...)"""
        it = srsgpu_rxq_item_t()
        for a, x in enumerate(td):
            it.td[a] = x.ctypes.data
        it.sf = sf
        for t, d in enumerate(data):
            it.data[t] = d.ctypes.data
        it.reset_softbuffer[0], it.reset_softbuffer[1] = reset
        return it

    def set_chest_cfg(self, average_subframe=False, noise_alg=0, smooth_filter_auto=False,
                      symbol_sz=None, rsrp_neighbour=False, cfo_enable=False, cfo_mask=0, gauss=None, filt=None):
        """the queue estimator's settings (srsgpu_chest_set_cfg on srsgpu_rxq_get_chest); gauss=(order, std)
        or filt (taps) sets the smoothing filter"""
        ch = _lib.srsgpu_rxq_get_chest(self.q)
        c = srsgpu_chest_cfg_t(int(average_subframe), noise_alg, int(smooth_filter_auto), int(rsrp_neighbour),
                               int(cfo_enable), cfo_mask, symbol_sz or symbol_sz_of(self.cell.nof_prb))
        if _lib.srsgpu_chest_set_cfg(ch, ctypes.byref(c)) != 0:
            raise RuntimeError("invalid chest configuration")
        if gauss is not None and _lib.srsgpu_chest_set_smooth_filter_gauss(ch, gauss[0], ctypes.c_float(gauss[1])) != 0:
            raise RuntimeError("invalid filter")
        if filt is not None:
            f = (ctypes.c_float * max(1, len(filt)))(*filt)
            if _lib.srsgpu_chest_set_smooth_filter(ch, f, len(filt)) != 0:
                raise RuntimeError("invalid filter")

    def decode(self, it):
        return _lib.srsgpu_rxq_decode(self.q, ctypes.byref(it))

    @staticmethod
    def ue_item(td, tti, rnti, data, tm=0, rnti_type=-1, softbuffer=(0, 1), ul_rnti=0, n_rb_ho=0, acks=(0, 0),
                feedback=0):
        """srsgpu_rxq_ue_dl_t: td complex64 arrays per rx antenna, data uint8 arrays per TB (both kept
        alive by the caller); feedback: FEEDBACK_CN | FEEDBACK_PMI"""
        u = srsgpu_rxq_ue_dl_t()
        u.feedback = feedback
        for a, x in enumerate(td):
            u.td[a] = x.ctypes.data
        u.tti, u.rnti, u.tm, u.rnti_type = tti, rnti, tm, rnti_type
        u.ul_rnti, u.n_rb_ho = ul_rnti, n_rb_ho
        u.acks[0], u.acks[1] = acks
        u.softbuffer[0], u.softbuffer[1] = softbuffer
        for t, d in enumerate(data):
            u.data[t] = d.ctypes.data
        return u

    def decode_rnti(self, u):
        return _lib.srsgpu_rxq_decode_rnti(self.q, ctypes.byref(u))

    def submit_ue_dl(self, u):
        t = ctypes.c_uint64(0)
        if _lib.srsgpu_rxq_submit_ue_dl(self.q, ctypes.byref(u), ctypes.byref(t)) != 0:
            raise RuntimeError("srsgpu_rxq_submit_ue_dl failed")
        return t.value

    def set_phich(self, length, resources):
        if _lib.srsgpu_rxq_set_phich(self.q, length, resources) != 0:
            raise RuntimeError("invalid PHICH configuration")

    def submit(self, it):
        t = ctypes.c_uint64(0)
        if _lib.srsgpu_rxq_submit(self.q, ctypes.byref(it), ctypes.byref(t)) != 0:
            raise RuntimeError("srsgpu_rxq_submit failed")
        return t.value

    def wait(self, ticket):
        return _lib.srsgpu_rxq_wait(self.q, ticket)

    def flush(self):
        _lib.srsgpu_rxq_flush(self.q)

    def timing(self):
        """srsgpu_rxq_timing: seconds per dispatcher stage so far"""
        v = (ctypes.c_double * 8)()
        _lib.srsgpu_rxq_timing(self.q, v, 8)
        names = ("front_end", "control", "grants", "pdsch_enqueue", "gpu_wait", "copy_out", "staging")
        return {k: v[i] for i, k in enumerate(names)}

    def drive(self, items, workers, reuse=0):
        """srsgpu_rxq_drive: native worker threads submit items (in index order per worker) while a
        collector waits for them; returns (t_sub, t_done, status) arrays"""
        import numpy as np
        n = len(items)
        ptrs = (ctypes.c_void_p * n)(*[ctypes.addressof(it) for it in items])
        t_sub, t_done = np.zeros(n), np.zeros(n)
        status = np.zeros(n, np.int32)
        if _lib.srsgpu_rxq_drive(self.q, ptrs, n, workers, reuse, t_sub.ctypes.data, t_done.ctypes.data,
                                 status.ctypes.data) != 0:
            raise RuntimeError("srsgpu_rxq_drive: a submission was refused")
        return t_sub, t_done, status

    def drive_paced(self, items, streams, depth, ticks, period_us=1000, workers=8):
        """srsgpu_rxq_drive_paced: `streams` streams submit one subframe each per period_us for `ticks`
        ticks, through items[(t % depth) * streams + s]; returns (latency_ms, status, acked, late_ms)"""
        import numpy as np
        assert len(items) == streams * depth
        ptrs = (ctypes.c_void_p * len(items))(*[ctypes.addressof(it) for it in items])
        lat = np.zeros(streams * ticks, np.float32)
        status = np.zeros(streams * ticks, np.int32)
        acked, late = ctypes.c_uint32(0), ctypes.c_double(0)
        if _lib.srsgpu_rxq_drive_paced(self.q, ptrs, streams, depth, ticks, period_us, workers, lat.ctypes.data,
                                       status.ctypes.data, ctypes.byref(acked), ctypes.byref(late)) != 0:
            raise RuntimeError("srsgpu_rxq_drive_paced: a submission was refused")
        return lat, status, acked.value, late.value

    def drive_paced_ex(self, items, streams, depth, ticks, period_us=1000, workers=8, cpus=()):
        """srsgpu_rxq_drive_paced_ex: drive_paced with the collector / producers pinned to `cpus` and the
        latency from the actual submission beside the latency from the tick; returns (latency_ms,
        submit_latency_ms, status, acked, late_ms)"""
        import numpy as np
        assert len(items) == streams * depth
        ptrs = (ctypes.c_void_p * len(items))(*[ctypes.addressof(it) for it in items])
        lat = np.zeros(streams * ticks, np.float32)
        slat = np.zeros(streams * ticks, np.float32)
        status = np.zeros(streams * ticks, np.int32)
        acked, late = ctypes.c_uint32(0), ctypes.c_double(0)
        cp = np.asarray(list(cpus), np.int32)
        if _lib.srsgpu_rxq_drive_paced_ex(self.q, ptrs, streams, depth, ticks, period_us, workers,
                                          cp.ctypes.data if cp.size else None, int(cp.size), lat.ctypes.data,
                                          slat.ctypes.data, status.ctypes.data, ctypes.byref(acked),
                                          ctypes.byref(late)) != 0:
            raise RuntimeError("srsgpu_rxq_drive_paced_ex: a submission was refused")
        return lat, slat, status, acked.value, late.value

    def set_affinity(self, cpus):
        """srsgpu_rxq_set_affinity: the queue's closer / dispatcher / completer threads onto `cpus`"""
        cp = np.asarray(list(cpus), np.int32)
        if _lib.srsgpu_rxq_set_affinity(self.q, cp.ctypes.data if cp.size else None, int(cp.size)) != 0:
            raise RuntimeError("srsgpu_rxq_set_affinity failed")

    def register(self, arr):
        """srsgpu_rxq_register: the GPU reads submissions whose samples lie in arr in place"""
        if _lib.srsgpu_rxq_register(self.q, arr.ctypes.data, arr.nbytes) != 0:
            raise RuntimeError("srsgpu_rxq_register failed")
        self._registered = getattr(self, "_registered", []) + [arr]

    def unregister(self, arr):
        if _lib.srsgpu_rxq_unregister(self.q, arr.ctypes.data) != 0:
            raise RuntimeError("srsgpu_rxq_unregister failed")
        self._registered = [a for a in self._registered if a is not arr]

    def alloc_host(self, shape, dtype):
        """srsgpu_rxq_alloc_host: a numpy array over queue-owned device-visible host memory (a zero-copy
        region of this queue, like a registered one). The array is invalid after free_host(arr) or
        close(): drop every reference to it (and its views) before either."""
        dt = np.dtype(dtype)
        nbytes = int(np.prod(shape)) * dt.itemsize
        p = _lib.srsgpu_rxq_alloc_host(self.q, max(nbytes, 1))
        if not p:
            raise RuntimeError("srsgpu_rxq_alloc_host failed")
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * max(nbytes, 1)).from_address(p))[:nbytes].view(dt).reshape(shape)
        self._owned = getattr(self, "_owned", {})
        self._owned[p] = nbytes
        return arr

    def free_host(self, arr):
        p = arr.ctypes.data
        if _lib.srsgpu_rxq_free_host(self.q, p) != 0:
            raise RuntimeError("srsgpu_rxq_free_host failed")
        self._owned.pop(p, None)

    SC16, CF32 = 1, 0

    def set_input_format(self, fmt, scale=0.0):
        if _lib.srsgpu_rxq_set_input_format(self.q, fmt, scale) != 0:
            raise RuntimeError("srsgpu_rxq_set_input_format failed")

    def ingest_stats(self):
        z, st = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _lib.srsgpu_rxq_ingest_stats(self.q, ctypes.byref(z), ctypes.byref(st))
        return z.value, st.value

    def stats(self):
        b, n = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _lib.srsgpu_rxq_stats(self.q, ctypes.byref(b), ctypes.byref(n))
        return b.value, n.value

    def close(self):
        if self.q:
            _lib.srsgpu_rxq_destroy(self.q)
            self.q = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def viterbi37_tb_decode_f_batch(torch, frames_sym, stream=None):
    """srsgpu_viterbi37_tb_decode_f_dev on a list of float32 symbol arrays (3F each): one launch,
    returns the decoded bits (one per byte) per frame"""
    offs, outs, so, oo = [], [], 0, 0
    for x in frames_sym:
        F = x.size // 3
        offs.append((so, oo, F))
        so += x.size
        oo += F
    arr = (srsgpu_viterbi_frame_t * len(offs))()
    for i, (a, b, F) in enumerate(offs):
        arr[i].sym_offset, arr[i].out_offset, arr[i].frame_length = a, b, F
    d_frames = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    d_sym = torch.from_numpy(np.concatenate(frames_sym).astype(np.float32)).cuda()
    d_out = torch.zeros(max(oo, 1), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    if _lib.srsgpu_viterbi37_tb_decode_f_dev(_vp(d_frames.data_ptr()), len(offs), _vp(d_sym.data_ptr()),
                                             _vp(d_out.data_ptr()), _vp(stream)) != 0:
        raise RuntimeError("srsgpu_viterbi37_tb_decode_f_dev failed")
    torch.cuda.synchronize()
    o = d_out.cpu().numpy()
    return [o[b:b + F].copy() for (_, b, F) in offs]


def dci_decode_batch(torch, cands, stream=None):
    """srsgpu_dci_decode_dev on a list of (float32 LLRs, nof_bits): one launch; returns per
    candidate (decoded, bits, crc_rem)"""
    arr = (srsgpu_dci_cand_t * len(cands))()
    lo, oo = 0, 0
    for i, (e, nb) in enumerate(cands):
        arr[i].llr_offset, arr[i].out_offset, arr[i].E, arr[i].nof_bits = lo, oo, e.size, nb
        lo += e.size
        oo += nb + 16
    d_c = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).cuda()
    d_llr = torch.from_numpy(np.concatenate([e for e, _ in cands]).astype(np.float32)).cuda()
    d_out = torch.zeros(oo, dtype=torch.uint8, device="cuda")
    d_crc = torch.zeros(len(cands), dtype=torch.int16, device="cuda")
    d_dec = torch.full((len(cands),), 7, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    if _lib.srsgpu_dci_decode_dev(_vp(d_c.data_ptr()), len(cands), _vp(d_llr.data_ptr()),
                                  _vp(d_out.data_ptr()), _vp(d_crc.data_ptr()), _vp(d_dec.data_ptr()),
                                  _vp(stream)) != 0:
        raise RuntimeError("srsgpu_dci_decode_dev failed")
    torch.cuda.synchronize()
    out, crc, dec = d_out.cpu().numpy(), d_crc.cpu().numpy().view(np.uint16), d_dec.cpu().numpy()
    res, oo = [], 0
    for i, (e, nb) in enumerate(cands):
        res.append((int(dec[i]), out[oo:oo + nb + 16].copy(), int(crc[i])))
        oo += nb + 16
    return res
