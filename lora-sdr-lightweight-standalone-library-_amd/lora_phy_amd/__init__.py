"""lora_phy_amd — MI355X-native LoRa PHY demod/mod hot path.

Python host layer over the C-ABI of include/lora_mi355x.h (liblora_mi355x.so, HIP
for gfx950).  IQ lives in torch.complex64 CUDA(HIP) tensors; the kernels run on the
current torch stream.  Host-side coding helpers (Hamming, Gray, interleave,
whitening, CRC) are in :mod:`lora_phy_amd.codes`; the phy.hpp-style functional API
is in :mod:`lora_phy_amd.phy`.
"""
from . import _capi, codes, iq_io, phy, shard  # noqa: F401
from ._capi import LoraError
from .demod import DemodPlan, DemodResult, LoRaDemod, compensate_offsets, spec_pipeline
from .mod import LoRaMod, modulate

__all__ = ["DemodPlan", "DemodResult", "LoRaDemod", "LoRaMod", "LoraError", "modulate",
           "compensate_offsets", "spec_pipeline", "codes", "iq_io", "phy", "shard", "lib_path", "version", "source_hash",
           "check_build"]


def lib_path() -> str:
    return _capi.LIB_PATH


def version() -> str:
    return _capi.lib().lora_version().decode()


def source_hash() -> str:
    """sha256 (16 hex digits) of the library sources in this tree, in the Makefile's order
    (csrc/*.hip, csrc/*.h, include/lora_mi355x.h, include/lora_mi355x_phy.hpp): equals the
    src= stamp of lora_version() iff the loaded library was built from these sources."""
    import glob
    import hashlib
    import os

    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    inc = os.path.join(os.path.dirname(pkg), "include")
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip"))) + sorted(glob.glob(os.path.join(pkg, "csrc", "*.h")))
    files += [os.path.join(inc, "lora_mi355x.h"), os.path.join(inc, "lora_mi355x_phy.hpp")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check_build() -> str:
    """Raise if the loaded liblora_mi355x.so was not built from this tree's sources."""
    v = version()
    want = source_hash()
    if f"src={want}" not in v:
        raise RuntimeError(f"{lib_path()} is stale: lora_version() = {v!r}, sources hash {want}; rebuild it")
    return v
