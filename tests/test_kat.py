"""The reference's turbo-code known-answer vectors (turbodecoder_test.h:76-103, extracted as data
by tests/golden/make_kat.py): 504 information bits and their 3 * 504 + 12 coded bits. CPU checks:
both encoders (the product's host encoder and the oracle) reproduce the coded bits, and the oracle
decodes the noiseless codeword. The GPU decode of the same vectors is in test_tdec_gpu.py.

One bit of the reference's KAT disagrees with the reference's own encoder: index 1512, the first
tail bit (x_K of the first constituent encoder's termination, turbocoder.c:160-177), is 0 in
known_data_encoded while srslte_tcod_encode, compiled from the reference's sources (oracle/_ref),
gives 1. The encoders here follow srslte_tcod_encode; the decoders take the KAT's bits as input,
as turbodecoder_test -k does (turbodecoder_test.c:237-240)."""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def kat():
    z = np.load(os.path.join(HERE, "golden", "tdec_kat.npz"))
    return z["known_data"], z["known_data_encoded"]


KAT_TAIL_MISMATCH = 1512  # see the module docstring


def _check_encoder(out, enc):
    diff = np.flatnonzero(out != enc)
    assert diff.tolist() == [KAT_TAIL_MISMATCH], diff
    assert out[KAT_TAIL_MISMATCH] == 1


def test_kat_product_encoder():
    import srsgpu_phy as s
    data, enc = kat()
    _check_encoder(s.Tcod(504).encode(data), enc)


def test_kat_oracle_encoder(oracle):
    data, enc = kat()
    _check_encoder(oracle.tcod_encode(data), enc)


def test_kat_tail_bit_is_the_reference_encoders():
    """the mismatching tail bit: the reference's own encoder (compiled from its sources) agrees
    with ours, not with its KAT"""
    from srsgpu_testlib import Ref, have_ref
    if not have_ref():
        import pytest
        pytest.skip("oracle/_ref not built (build container only)")
    data, enc = kat()
    _check_encoder(Ref().tcod_encode(data), enc)


def test_kat_oracle_noiseless_decode(oracle):
    from srsgpu_testlib import AUTO, GENERIC, SSE, SSE_WINDOW, pack_bits
    data, enc = kat()
    llr = np.where(enc == 1, 100, -100).astype(np.int16)
    for impl in (AUTO, GENERIC, SSE, SSE_WINDOW):
        dec, _, _ = oracle.tdec_run(impl, 0, llr, 504, 8)
        assert (dec[-1] == pack_bits(data)).all(), impl
