"""Register, scratch and LDS-banking guards for the pipeline kernels (CPU: code-object
metadata of the built library and the LDS bank model - no GPU needed).

* The benchmarked pipeline kernels keep no scratch (spills) and fit the register budget
  that gives them their occupancy: a regression here shows up
  on the GPU only as a slower step.
* The SF7 LDS slot map (lora_demod_fast.hip LdsMap<7>) is conflict-free for every access
  of the symbol pass under the MI355X banking rules (tools/lds/lds_sim.py).
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "tools", "lds"))
LIB = os.path.join(ROOT, "lora-sdr-lightweight-standalone-library-_amd", "lora_phy_amd", "lib", "liblora_mi355x.so")
SRC = os.path.join(ROOT, "lora-sdr-lightweight-standalone-library-_amd", "csrc", "lora_demod_fast.hip")


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    import kernel_resources

    if not os.path.exists(kernel_resources.READELF):
        pytest.skip("llvm-readelf not available")
    rows = kernel_resources.kernels(LIB)
    out = {}
    for r in rows:
        m = re.search(r"(k_\w+(<[^>]*>)?)", r.get("demangled", r["name"]))
        if m:
            out.setdefault(m.group(1), r)
    return out


# (kernel, max VGPRs): the speculative pipeline of the bench workloads (SF7, SF12, osr 2, API)
PIPELINE = [
    ("k_est_split<7, 0>", 128),
    ("k_spec_demod<7, 0, false, 1, 0>", 128),
    ("k_cert_split<7, 0>", 128),
    ("k_spec_fix<7, 0>", 256),
    ("k_est_fast<12, 0, 1>", 128),
    ("k_spec_demod<12, 0, false, 1, 0>", 128),
    ("k_est_fast<12, 0, 2>", 128),
    ("k_spec_fix<12, 0>", 256),
    ("k_est_fast<7, 2, 1>", 256),
    ("k_spec_demod<7, 0, false, 2, 0>", 128),
    ("k_est_fast<7, 2, 2>", 256),
    # the API line (LORA_MODE_API through the pipeline): exact estimate, symbol pass, stage 2
    ("k_est_fast<7, 2, 0>", 256),
    ("k_spec_demod<7, 0, false, 1, 1>", 128),
    # the RAW line (the detector alone through the pipeline)
    ("k_spec_demod<7, 0, false, 1, 2>", 128),
    ("k_cert_raw<7>", 128),
]


@pytest.mark.parametrize("name,max_vgpr", PIPELINE)
def test_pipeline_kernel_has_no_scratch(kernels, name, max_vgpr):
    assert name in kernels, sorted(k for k in kernels if k.startswith(name.split("<")[0]))
    r = kernels[name]
    assert r.get("private_segment_fixed_size", 0) == 0, (name, r)
    assert r.get("vgpr_spill_count", 0) == 0, (name, r)
    assert r["vgpr_count"] <= max_vgpr, (name, r["vgpr_count"])


def _lds_map(sf):
    """LdsMap<sf> weights (W3, W[], PAD) parsed from the kernel source."""
    src = open(SRC).read()
    i = src.index("template <> struct LdsMap<%d>" % sf)
    body = src[i:src.index("template", i + 8)]  # up to the next specialisation
    w3 = re.search(r"W3 = (\d+)", body)
    w = [int(x) for x in re.search(r"W\[\d+\] = \{([^}]*)\}", body).group(1).split(",")]
    pad = int(re.search(r"PAD = (\d+)", body).group(1))
    return (int(w3.group(1)) if w3 else 0), w, pad


def test_sf7_lds_map_is_conflict_free_for_the_symbol_pass():
    from lds_sim import geo, patterns

    sf = 7
    w3, w, pad = _lds_map(sf)
    g = geo(sf)

    def slot(p):
        return p + ((p >> 3) & 1) * w3 + sum(((p >> (4 + i)) & 1) * wi for i, wi in enumerate(w))

    slots = [slot(p) for p in range(g["N"])]
    assert len(set(slots)) == g["N"]  # injective
    rowc = g["N"] + w3 + sum(w) + pad

    def degree(s, gsz, nb):
        worst = 1
        for i in range(0, 64, gsz):
            banks = {}
            for v in set(s[i:i + gsz]):
                for d in (2 * v, 2 * v + 1):
                    banks.setdefault(d % nb, set()).add(d)
            worst = max(worst, max(len(x) for x in banks.values()))
        return worst

    for name, pat in patterns(sf):
        s = [gg * rowc + slot(p) for gg, p in pat]
        if name.startswith("w"):  # pass-1 write-back: ds_write_b64 / ds_write2_b64, 16-lane groups
            assert degree(s, 16, 32) == 1, name
        elif name.startswith("r"):  # pass-A reads as ds_read_b64 (32 lanes) and ds_read2_b64 (16)
            assert degree(s, 32, 64) == 1, name
            assert degree(s, 16, 32) == 1, name
