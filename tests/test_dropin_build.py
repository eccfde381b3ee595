"""CPU: the C++ drop-in builds and links - include/lora_mi355x_phy.hpp compiles for a caller
that includes the reference's header names (include/compat), and the programs the GPU
tests run resolve every lora_phy:: symbol from liblora_mi355x.so."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB = os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd", "lora_phy_amd", "lib", "liblora_mi355x.so")
E2E = os.path.join(HERE, "native", "e2e_dropin")


def test_dropin_header_compiles_for_reference_style_caller(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    src = tmp_path / "caller.cpp"
    src.write_text(
        "#include <lora_phy/phy.hpp>\n#include <lora_phy/ChirpGenerator.hpp>\n#include <vector>\n"
        "int main(){ lora_phy::lora_demod_workspace ws{}; std::vector<std::complex<float>> s(512), d(128);\n"
        " float ph=0; genChirp(d.data(),128,1,128,0.0f,true,1.0f,ph,lora_phy::bw_scale(lora_phy::bandwidth::bw_125));\n"
        " uint16_t out[4]; uint8_t sync=0;\n"
        " lora_phy::lora_demod_init(&ws,7,lora_phy::window_type::window_none,s.data(),s.size());\n"
        " size_t n=lora_phy::lora_demodulate(&ws,s.data(),s.size(),out,1,&sync); lora_phy::lora_demod_free(&ws);\n"
        " return (int)n + ws.metrics.crc_ok; }\n")
    r = subprocess.run(["g++", "-std=c++11", "-fsyntax-only", "-I", os.path.join(REPO, "include", "compat"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_dropin_symbols_exported():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    out = subprocess.run(["nm", "-DC", LIB], capture_output=True, text=True).stdout
    for sym in ("lora_phy::lora_demod_init(", "lora_phy::lora_demod_free(", "lora_phy::lora_demodulate(",
                "lora_phy::lora_modulate(", "lora_phy::lora_encode(", "lora_phy::lora_decode(", "genChirp("):
        assert any(sym in line and " T " in line for line in out.splitlines()), sym


def test_e2e_program_links():
    if not os.path.exists(E2E):
        pytest.skip("tests/native/e2e_dropin not built")
    r = subprocess.run(["ldd", E2E], capture_output=True, text=True)
    assert "liblora_mi355x.so" in r.stdout and "not found" not in r.stdout, r.stdout
