"""Record golden PDCCH receptions and DCI unpackings from the reference build (`make -C oracle ref`):

  - the PDCCH symbol order (srslte_regs_init + srslte_regs_pdcch_get, regs.c) and NOF_CCE for each
    cell and CFI;
  - control regions built with srslte_pdcch_encode (pdcch.c:568-643) through a synthetic channel
    (tests/srsgpu_testlib.py pdcch_subframe), their srslte_pdcch_extract_llr_multi LLRs
    (pdcch.c:424-506), and the reference's own ue_dl.c searches run by oracle/_ref/ref_front:
    srslte_ue_dl_find_dl_dci(_type) for C-, SI- and RA-RNTIs, then srslte_ue_dl_find_ul_dci for the
    C-RNTI (ue_dl.c:768-932, phch_worker's order) with srslte_dci_msg_to_ul_grant of a found UL DCI;
  - srslte_dci_msg_to_dl_grant (dci.c:49-90 with ra.c) of the found messages and of random
    messages of every DL format.

    python tests/golden/make_pdcch_golden.py   -> tests/golden/pdcch_golden.npz
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from srsgpu_testlib import (F1, F1A, F1B, F1C, F1D, F2, F2A, F2B, Ref, dci_sizeof_ref,  # noqa: E402
                            dci_to_dl_grant_ref, dci_to_ul_grant_ref, find_dci_ref, pdcch_llr, pdcch_locations,
                            pdcch_map, pdcch_subframe, random_dl_msg, random_ul_msg)


def main():
    ref = Ref()
    rng = np.random.default_rng(2018)
    arrays, cases, maps, grants, ulgrants = {}, [], [], [], []
    # symbol orders
    for nof_prb in (6, 15, 25, 50, 75, 100):
        for cell_id in (0, 7, 301):
            for nports in (1, 2):
                pl, pr = int(rng.integers(0, 2)), int(rng.integers(0, 4))
                for cfi in (1, 2, 3):
                    idx, ncce = pdcch_map(ref, nof_prb, cell_id, nports, pl, pr, cfi, ref=True)
                    key = "m%d" % len(maps)
                    arrays[key] = idx
                    maps.append(dict(key=key, nof_prb=nof_prb, cell_id=cell_id, nports=nports, phich_len=pl,
                                     phich_res=pr, cfi=cfi, nof_cce=ncce))
    # received subframes; the "batch" group shares one cell for the multi-subframe launches
    cells = [(p, c, np_, nr) for p in (6, 15, 25, 50, 100) for c in (int(rng.integers(0, 504)),)
             for np_ in (1, 2) for nr in (1, 2)]
    groups = [("single", cell, 1 if cell[0] >= 50 else 2) for cell in cells] + [("batch", (25, 77, 2, 2), 6)]
    groups += [("refused", (110, 5, 2, 1), 2)]  # 96 CCEs: UE spaces reaching nCCE 88 end in an error
    for group, (nof_prb, cell_id, nports, nrx), reps in groups:
        pl, pr = (int(rng.integers(0, 2)), int(rng.integers(0, 4))) if group != "refused" else (0, 0)
        for r in range(reps):
            cfi, sf_idx, tm = int(rng.integers(1, 4)), int(rng.integers(0, 10)), int(rng.integers(0, 8))
            if group == "refused":
                cfi = 3
            y, h, searches, noise = pdcch_subframe(ref, rng, nof_prb, cell_id, nports, nrx, pl, pr, cfi,
                                                   sf_idx, tm, snr_db=float(rng.choice([6.0, 12.0, 30.0])))
            if group == "refused":  # C-RNTIs whose UE-specific space holds a location past nCCE 87
                ncce = pdcch_map(ref, nof_prb, cell_id, nports, pl, pr, cfi, ref=True)[1]
                hits = [x for x in range(0x100, 0x2000)
                        if any(c > 87 for _, c in pdcch_locations(ref, ncce, sf_idx, x, False))]
                searches += [(x, tm, -1, x) for x in hits[:4]] + [(x, tm, 0, x) for x in hits[4:6]]
            nre = (cfi + (1 if nof_prb <= 10 else 0)) * 12 * nof_prb  # store the control symbols only
            y = [v[:nre] for v in y]
            h = [[v[:nre] for v in hp] for hp in h]
            llr = pdcch_llr(ref, nof_prb, cell_id, nports, pl, pr, nrx, cfi, sf_idx, noise, y, h, ref=True)
            llr2, found = find_dci_ref(nof_prb, cell_id, nports, nrx, pl, pr, cfi, sf_idx, noise, y, h, searches)
            assert np.array_equal(llr.view(np.uint32), llr2.view(np.uint32))
            key = "c%d" % len(cases)
            for a in range(nrx):
                arrays["%s_y%d" % (key, a)] = y[a]
                for p in range(nports):
                    arrays["%s_h%d%d" % (key, p, a)] = h[p][a]
            arrays[key + "_llr"] = llr
            res = []
            for j, ((rnti, stm, rtype, ul_rnti), (dl, ul, ulg)) in enumerate(zip(searches, found)):
                found_, fmt, L, ncce, nb, bits = dl
                arrays["%s_s%d_bits" % (key, j)] = bits
                arrays["%s_s%d_ulbits" % (key, j)] = ul[5]
                res.append(dict(rnti=rnti, tm=stm, rnti_type=rtype, found=found_, format=fmt, L=L, ncce=ncce,
                                nof_bits=nb, ul_rnti=ul_rnti, ul_found=ul[0], ul_format=ul[1], ul_L=ul[2],
                                ul_ncce=ul[3], ul_nof_bits=ul[4], ul_grant_ret=ulg[0],
                                ul_dci=[int(v) for v in ulg[1]], ul_grant=[int(v) for v in ulg[2]]))
                if found_ > 0:
                    grants.append((bits, fmt, rnti, nof_prb, nports, nb))
                if ul[0] > 0:
                    ulgrants.append((ul[5][:ul[4]], nof_prb))
            cases.append(dict(key=key, group=group, nof_prb=nof_prb, cell_id=cell_id, nports=nports, nrx=nrx,
                              phich_len=pl, phich_res=pr, cfi=cfi, sf_idx=sf_idx, noise=noise,
                              searches=res))
    # DCI unpacking: the found messages and random ones of every DL format / RNTI kind
    for nof_prb in (6, 15, 25, 50, 75, 100):
        for nports in (1, 2):
            for fmt in (F1, F1A, F1C, F1B, F1D, F2, F2A, F2B):
                for k in range(4):
                    rnti = [0x4601, 0xFFFF, 0x0003, 0xFFFE][k]
                    if k < 2:
                        b = random_dl_msg(ref, rng, fmt, nof_prb, nports, crc_is_crnti=(k == 0))
                    else:
                        b = rng.integers(0, 2, dci_sizeof_ref(ref, fmt, nof_prb, nports)).astype(np.uint8)
                    grants.append((b, fmt, rnti, nof_prb, nports, len(b)))
    gman = []
    for i, (b, fmt, rnti, nof_prb, nports, nb) in enumerate(grants):
        r, d, g, p = dci_to_dl_grant_ref(ref, b, fmt, rnti, nof_prb, nports, nof_bits=nb)
        key = "g%d" % i
        arrays[key + "_bits"] = np.asarray(b, np.uint8)
        arrays[key + "_prb"] = p
        gman.append(dict(key=key, format=fmt, rnti=rnti, nof_prb=nof_prb, nports=nports, nof_bits=nb, ret=r,
                         dci=[int(v) for v in d], grant=[int(v) for v in g]))
    # format 0 unpacking: the found UL messages and random reference-packed ones, with and without a
    # PUSCH hopping offset
    for nof_prb in (6, 15, 25, 50, 75, 100):
        for k in range(10):
            ulgrants.append((random_ul_msg(ref, rng, nof_prb, hop_p=0.6), nof_prb))
    ugman = []
    for i, (b, nof_prb) in enumerate(ulgrants):
        for n_rb_ho in (0, 4):
            r, d, g = dci_to_ul_grant_ref(ref, b, nof_prb, n_rb_ho)
            key = "u%d_%d" % (i, n_rb_ho)
            arrays[key + "_bits"] = np.asarray(b, np.uint8)
            ugman.append(dict(key=key, nof_prb=nof_prb, n_rb_ho=n_rb_ho, nof_bits=len(b), ret=r,
                              dci=[int(v) for v in d], grant=[int(v) for v in g]))
    # 4 CRS ports (a separate stream, after everything above): symbol orders and received subframes,
    # transmit diversity over the REG quadruplets (precoding.c:388-423 via pdcch.c:495-496)
    rng4 = np.random.default_rng(4444)
    for nof_prb in (6, 25, 100):
        for cfi in (1, 2, 3):
            cell_id = int(rng4.integers(0, 504))
            pl, pr = int(rng4.integers(0, 2)), int(rng4.integers(0, 4))
            idx, ncce = pdcch_map(ref, nof_prb, cell_id, 4, pl, pr, cfi, ref=True)
            key = "m%d" % len(maps)
            arrays[key] = idx
            maps.append(dict(key=key, nof_prb=nof_prb, cell_id=cell_id, nports=4, phich_len=pl, phich_res=pr,
                             cfi=cfi, nof_cce=ncce))
    for nof_prb, nrx in ((6, 1), (15, 2), (25, 1), (50, 2), (100, 2), (100, 1)):
        cell_id = int(rng4.integers(0, 504))
        pl, pr = int(rng4.integers(0, 2)), int(rng4.integers(0, 4))
        for r in range(2):
            cfi, sf_idx, tm = int(rng4.integers(1, 4)), int(rng4.integers(0, 10)), int(rng4.integers(0, 8))
            y, h, searches, noise = pdcch_subframe(ref, rng4, nof_prb, cell_id, 4, nrx, pl, pr, cfi, sf_idx, tm,
                                                   snr_db=float(rng4.choice([6.0, 12.0, 30.0])))
            nre = (cfi + (1 if nof_prb <= 10 else 0)) * 12 * nof_prb
            y = [v[:nre] for v in y]
            h = [[v[:nre] for v in hp] for hp in h]
            llr = pdcch_llr(ref, nof_prb, cell_id, 4, pl, pr, nrx, cfi, sf_idx, noise, y, h, ref=True)
            llr2, found = find_dci_ref(nof_prb, cell_id, 4, nrx, pl, pr, cfi, sf_idx, noise, y, h, searches)
            assert np.array_equal(llr.view(np.uint32), llr2.view(np.uint32))
            key = "c%d" % len(cases)
            for a in range(nrx):
                arrays["%s_y%d" % (key, a)] = y[a]
                for p in range(4):
                    arrays["%s_h%d%d" % (key, p, a)] = h[p][a]
            arrays[key + "_llr"] = llr
            res = []
            for j, ((rnti, stm, rtype, ul_rnti), (dl, ul, ulg)) in enumerate(zip(searches, found)):
                found_, fmt, L, ncce, nb, bits = dl
                arrays["%s_s%d_bits" % (key, j)] = bits
                arrays["%s_s%d_ulbits" % (key, j)] = ul[5]
                res.append(dict(rnti=rnti, tm=stm, rnti_type=rtype, found=found_, format=fmt, L=L, ncce=ncce,
                                nof_bits=nb, ul_rnti=ul_rnti, ul_found=ul[0], ul_format=ul[1], ul_L=ul[2],
                                ul_ncce=ul[3], ul_nof_bits=ul[4], ul_grant_ret=ulg[0],
                                ul_dci=[int(v) for v in ulg[1]], ul_grant=[int(v) for v in ulg[2]]))
            cases.append(dict(key=key, group="ports4", nof_prb=nof_prb, cell_id=cell_id, nports=4, nrx=nrx,
                              phich_len=pl, phich_res=pr, cfi=cfi, sf_idx=sf_idx, noise=noise, searches=res))
            for j, (rnti, _, _, _) in enumerate(searches):  # the found messages' grants, 4-port unpacking
                found_, fmt, _, _, nb, bits = found[j][0]
                if found_ > 0:
                    r_, d, g, p = dci_to_dl_grant_ref(ref, bits, fmt, rnti, nof_prb, 4, nof_bits=nb)
                    gkey = "g%d" % len(gman)
                    arrays[gkey + "_bits"] = np.asarray(bits, np.uint8)
                    arrays[gkey + "_prb"] = p
                    gman.append(dict(key=gkey, format=fmt, rnti=rnti, nof_prb=nof_prb, nports=4, nof_bits=nb,
                                     ret=r_, dci=[int(v) for v in d], grant=[int(v) for v in g]))
    man = dict(maps=maps, cases=cases, grants=gman, ul_grants=ugman)
    arrays["manifest"] = np.frombuffer(json.dumps(man).encode(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "pdcch_golden.npz"), **arrays)
    nf = sum(s["found"] > 0 for c in cases for s in c["searches"])
    ne = sum(s["found"] < 0 for c in cases for s in c["searches"])
    nu = sum(s["ul_found"] > 0 for c in cases for s in c["searches"])
    print("maps %d, subframes %d, searches found %d (refused %d) of %d, UL found %d, grants %d (ok %d), "
          "UL grants %d (ok %d)" % (len(maps), len(cases), nf, ne, sum(len(c["searches"]) for c in cases), nu,
                                    len(gman), sum(g["ret"] == 0 for g in gman), len(ugman),
                                    sum(g["ret"] == 0 for g in ugman)))


if __name__ == "__main__":
    main()
