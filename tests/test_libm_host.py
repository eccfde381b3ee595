"""CPU: the device libm ports (csrc/lora_libm.h) equal this host's glibc bit for bit.

The reference's outputs depend on glibc's sincosf / atan2f / hypotf / log10f (see the
header of lora_libm.h); the kernels evaluate the same algorithms.  This builds
tests/native/libm_check.cpp with g++ and compares over a strided sweep of all 2^32
float bit patterns for sincosf (and its branch-free fast-path forms over |y| < 120),
and a hashed sample for the others.  An exhaustive sweep is `libm_check 1 <threads>`.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "libm_check.cpp")
BIN = os.path.join(HERE, "native", "libm_check")


@pytest.fixture(scope="module")
def results():
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(
            os.path.getmtime(SRC),
            os.path.getmtime(os.path.join(HERE, "..", "lora-sdr-lightweight-standalone-library-_amd",
                                          "csrc", "lora_libm.h"))):
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-o", BIN, SRC,
                               "-lm", "-lpthread"])
    out = subprocess.run([BIN, "61", str(min(8, os.cpu_count() or 1))], capture_output=True,
                         text=True, check=True, timeout=600).stdout
    res = {}
    for line in out.splitlines():
        name, n, bad = line.split()
        res[name] = (int(n), int(bad))
    return res


@pytest.mark.parametrize("name", ["sincosf", "sincosf_bf", "sincosf_large", "sincosf_fast", "sincosf_fast_k", "sincosf_fast_k_nz",
                                  "atan2f", "hypotf", "logf", "log10f"])
def test_bit_exact_vs_glibc(results, name):
    n, bad = results[name]
    assert n > 1_000_000
    assert bad == 0, f"{name}: {bad} of {n} differ from glibc"
