"""lora_phy_amd — MI355X-native LoRa PHY demod/mod hot path.

Python host layer over the C-ABI of include/lora_mi355x.h (liblora_mi355x.so, HIP
for gfx950).  IQ lives in torch.complex64 CUDA(HIP) tensors; the kernels run on the
current torch stream.  Host-side coding helpers (Hamming, Gray, interleave,
whitening, CRC) are in :mod:`lora_phy_amd.codes`; the phy.hpp-style functional API
is in :mod:`lora_phy_amd.phy`.
"""
from . import _capi, codes, iq_io, phy, shard  # noqa: F401
from ._capi import LoraError
from .demod import DemodPlan, DemodResult, LoRaDemod, compensate_offsets
from .mod import LoRaMod, modulate

__all__ = ["DemodPlan", "DemodResult", "LoRaDemod", "LoRaMod", "LoraError", "modulate",
           "compensate_offsets", "codes", "iq_io", "phy", "shard", "lib_path", "version"]


def lib_path() -> str:
    return _capi.LIB_PATH


def version() -> str:
    return _capi.lib().lora_version().decode()
