"""Extracts the reference's turbo-code known-answer vectors as data: known_data (504 bits) and
known_data_encoded (3 * 504 + 12 coded bits) from
/root/reference/lib/src/phy/fec/test/turbodecoder_test.h:76-103 (the arrays the reference's
turbodecoder_test -k decodes), into tests/golden/tdec_kat.npz. Run in the build container only
(the reference does not exist on the GPU box); the .npz is the committed fixture."""
import os
import re

import numpy as np

SRC = "/root/reference/lib/src/phy/fec/test/turbodecoder_test.h"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tdec_kat.npz")


def array(text, name):
    m = re.search(r"\b%s\s*\[[^\]]*\]\s*=\s*\{([^}]*)\}" % re.escape(name), text)
    return np.array([int(v) for v in m.group(1).replace("\n", " ").split(",") if v.strip()], np.uint8)


def main():
    text = open(SRC).read()
    data, enc = array(text, "known_data"), array(text, "known_data_encoded")
    errs = np.array([int(v) for v in re.search(r"known_data_errors\[4\]\s*=\s*\{([^}]*)\}", text)
                     .group(1).split(",")], np.int32)
    ebno = float(re.search(r"#define KNOWN_DATA_EBNO\s+([0-9.]+)", text).group(1))
    assert data.size == 504 and enc.size == 3 * 504 + 12
    np.savez_compressed(OUT, known_data=data, known_data_encoded=enc, known_data_errors=errs,
                        known_data_ebno=np.float32(ebno))
    print("wrote", OUT, data.size, enc.size, errs.tolist(), ebno)


if __name__ == "__main__":
    main()
