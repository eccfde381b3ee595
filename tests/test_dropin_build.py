"""CPU: the C++ drop-in builds and links - include/lora_mi355x_phy.hpp compiles for a caller
that includes the reference's header names (include/compat), and the programs the GPU
tests run resolve every lora_phy:: symbol from liblora_phy.so (the drop-in library over
liblora_mi355x.so)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
LIB = os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd", "lora_phy_amd", "lib", "liblora_phy.so")
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
                "lora_phy::lora_modulate(", "lora_phy::lora_encode(", "lora_phy::lora_decode(", "genChirp(",
                # the workspace API (phy.hpp:102-156)
                "lora_phy::init(", "lora_phy::reset(", "lora_phy::encode(", "lora_phy::decode(",
                "lora_phy::modulate(", "lora_phy::demodulate(", "lora_phy::estimate_offsets(",
                "lora_phy::compensate_offsets(", "lora_phy::get_last_metrics(", "lora_phy::detail::release(",
                "lora_phy_dropin_status"):
        assert any(sym in line and " T " in line for line in out.splitlines()), sym


def test_e2e_program_links():
    if not os.path.exists(E2E):
        pytest.skip("tests/native/e2e_dropin not built")
    r = subprocess.run(["ldd", E2E], capture_output=True, text=True)
    assert "liblora_phy.so" in r.stdout and "liblora_mi355x.so" in r.stdout and "not found" not in r.stdout, r.stdout


def test_workspace_api_compiles_for_rx_runner_style_caller(tmp_path):
    """runners/rx_runner.cpp:93-122's use of the workspace API (C++11, the reference's
    standard) against include/compat."""
    if not shutil.which("g++"):
        pytest.skip("no g++")
    src = tmp_path / "rx.cpp"
    src.write_text(
        "#include <lora_phy/phy.hpp>\n#include <vector>\nusing namespace lora_phy;\n"
        "int main(){ std::vector<uint16_t> symbols(8); std::vector<std::complex<float>> fft_in(128), fft_out(128),\n"
        " samples(1280);\n lora_params params{}; params.sf = 7; params.bw = bandwidth::bw_125; params.cr = 1;\n"
        " lora_workspace ws{}; ws.symbol_buf = symbols.data(); ws.fft_in = fft_in.data(); ws.fft_out = fft_out.data();\n"
        " if (init(&ws, &params) != 0) return 1;\n"
        " ssize_t n = demodulate(&ws, samples.data(), samples.size(), symbols.data(), symbols.size());\n"
        " std::vector<uint8_t> decoded(4); ssize_t b = decode(&ws, symbols.data(), n, decoded.data(), decoded.size());\n"
        " const lora_metrics* m = get_last_metrics(&ws); estimate_offsets(&ws, samples.data(), samples.size());\n"
        " compensate_offsets(&ws, samples.data(), samples.size()); reset(&ws);\n"
        " return (int)(b + (m->crc_ok ? 1 : 0)); }\n")
    r = subprocess.run(["g++", "-std=c++11", "-fsyntax-only", "-I", os.path.join(REPO, "include", "compat"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
