"""CPU: the closed-form frequency runs of genChirp (csrc/lora_chirp.h) behind the
modulator's frame kernel k_mod_frame are exact.

tests/native/chirp_seg_check.cpp (built here with g++) walks every configuration
lora_modulate gives genChirp (SF 2-12, osr 1-4, 125/250/500 kHz; every symbol < N, every
sync nibble, and a sample of uint16 codewords >= N) and compares each run-evaluated
frequency with the recurrence of ChirpGenerator.hpp:118-120 bit for bit - about 9e8 steps.
The run count of every symbol < N stays within the kernel's table (chirp_seg_cap); larger
values may exceed it, and the kernel then runs that chirp's recurrence itself.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "chirp_seg_check.cpp")
HDR = os.path.join(HERE, "..", "lora-sdr-lightweight-standalone-library-_amd", "csrc", "lora_chirp.h")
BIN = os.path.join(HERE, "native", "chirp_seg_check")


def test_chirp_runs_equal_the_recurrence():
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        subprocess.check_call(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-o", BIN, SRC])
    r = subprocess.run([BIN, "12", "1"], capture_output=True, text=True, timeout=300)
    rows = [list(map(int, line.split())) for line in r.stdout.splitlines()]
    assert len(rows) == 11 * 4, r.stdout + r.stderr
    for sf, osr, chirps, steps, bad, max_runs, cap, over in rows:
        assert bad == 0, f"SF{sf} osr {osr}: {bad} mismatches"
        assert steps > 0 and max_runs <= cap
    assert r.returncode == 0
