"""Register / scratch budget of the PDSCH front-end kernels (CPU: a cross-compile of
empower-srslte_amd/csrc/pdsch_kernels.hip for gfx950 with the compiler's resource-usage remarks).

A run-time index into a kernel's local descriptor (say the item's port planes by a computed pair
index) makes the compiler keep the whole descriptor in scratch memory: in round 4 that took
k_pdsch_llr from 63 to 155 us per 512 subframes (DESIGN §5 "Front end (round 4)"). This guards it."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _usage(src):
    """{kernel (mangled): {"VGPRs": n, "ScratchSize": n, ...}} from -Rpass-analysis=kernel-resource-usage"""
    out = subprocess.run([HIPCC, "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                          "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(REPO, "empower-srslte_amd", "csrc"),
                          "-c", src, "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = res.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    return res


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_pdsch_kernels_keep_descriptors_in_registers():
    u = _usage(os.path.join(REPO, "empower-srslte_amd", "csrc", "pdsch_kernels.hip"))
    names = {k: v for k, v in u.items() if re.search(r"k_pdsch_llr|k_pdcch_llr|k_csi_correct|k_gold", k)}
    assert len(names) >= 4, list(u)
    for k, v in names.items():
        assert v.get("ScratchSize", 0) == 0, (k, v)
        assert v.get("VGPRs", 0) <= 128, (k, v)  # 4+ waves per SIMD
