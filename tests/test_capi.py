"""CPU: the C-ABI library loads, exports exactly what include/lora_mi355x.h declares,
carries gfx950 code, and rejects bad parameters before touching the GPU.

No compute call is made here (there is no GPU in the build container); the parity
tests proper are the `-m gpu` ones.
"""
import ctypes as C
import os
import re
import subprocess

import pytest

from lora_phy_amd import _capi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "lora_mi355x.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(lora_\w+)\s*\(", text, flags=re.M)))


def test_header_matches_binding_table():
    assert declared_functions() == sorted(_capi.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = _capi.lib()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = set(declared_functions()) - exported
    assert not missing, missing


def test_library_carries_gfx950_code_object():
    blob = open(_capi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"__hip_fatbin" in blob or b"HIPF" in blob or b".hip_fatbin" in blob


def test_version_and_error_string():
    lib = _capi.lib()
    assert lib.lora_version().decode().startswith("lora_mi355x")
    assert isinstance(lib.lora_last_error(), bytes)


@pytest.mark.parametrize("field,value", [("sf", 1), ("sf", 13), ("bw_hz", 100000), ("window", 7),
                                         ("mode", 9), ("osr", 1000), ("precision", 2), ("precision", -1)])
def test_plan_create_rejects_bad_parameters(field, value):
    """Validation happens before any HIP call: -EINVAL (reference returns -1,
    phy.cpp:27-33), with a message."""
    lib = _capi.lib()
    prm = _capi.DemodParams(7, 1, 125000, 0, 0, 0, 0)
    setattr(prm, field, value)
    h = C.c_void_p()
    rc = lib.lora_demod_plan_create(C.byref(prm), C.byref(h))
    assert rc == _capi.LORA_EINVAL
    assert lib.lora_last_error().decode()
    with pytest.raises(_capi.LoraError):
        _capi.check(rc)


def test_param_structs_match_header():
    """The ctypes mirrors of lora_demod_params / lora_demod_outputs list the header's
    fields in the header's order (a drift would silently shift every field after it)."""
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for cname, pystruct in (("lora_demod_params", _capi.DemodParams), ("lora_demod_outputs", _capi.DemodOutputs)):
        body = re.search(r"typedef struct \{([^}]*)\}\s*" + cname + ";", text).group(1)
        fields = re.findall(r"(\w+)\s*;", body)
        assert fields == [f for f, _ in pystruct._fields_], cname


def test_null_arguments_rejected():
    lib = _capi.lib()
    assert lib.lora_demod_plan_create(None, None) == _capi.LORA_EINVAL
    assert lib.lora_demod_plan_destroy(None) in (_capi.LORA_OK, _capi.LORA_EINVAL)
    assert lib.lora_demod_batch(None, None, 0, 0, 0, None, None, 0, None) == _capi.LORA_EINVAL


def test_product_path_has_no_cpu_fallback():
    import torch

    import lora_phy_amd as amd

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        amd.DemodPlan(7)
    with pytest.raises(TypeError):
        amd.modulate(torch.zeros(4, dtype=torch.int32), 7)


def test_library_built_from_these_sources():
    """lora_version()'s src= stamp equals the hash of the sources in this tree (a stale
    prebuilt liblora_mi355x.so would fail here and in smoke())."""
    import lora_phy_amd

    v = lora_phy_amd.check_build()
    assert "git=" in v and "(gfx950)" in v


def test_lora_demod_thresh_and_mtu_validation():
    """Pothos-only parameters (examples/lora_simulation.pth:440,444): thresh has no gate in
    the reference path, so a non-default value raises instead of being ignored; mtu >= 1."""
    import pytest as _pytest

    import lora_phy_amd

    with _pytest.raises(ValueError):
        lora_phy_amd.LoRaDemod(7, thresh=-20.0)
    with _pytest.raises(ValueError):
        lora_phy_amd.LoRaDemod(7, mtu=0)


def test_sf7_pair_load_positions():
    """k_spec_demod's SF7 pair-load pass (PL) writes residue r's pass-1 group to position
    rev[r] >> 3 computed as 4 (r & 3) + (r >> 2): kissfft's leaf order at N = 128 (radices
    4, 4, 4, 2; tools/lds/lds_sim.leaf_rev, the design aid's replica of the device table)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "lds"))
    import lds_sim

    rev = lds_sim.leaf_rev(128)
    assert all(rev[r] >> 3 == ((r & 3) << 2) | (r >> 2) for r in range(16))
