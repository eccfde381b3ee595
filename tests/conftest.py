"""pytest configuration: markers and import paths.

`-m gpu` tests run the HIP path on a real MI355X and compare it with the CPU oracle
(oracle/, test infrastructure) and the committed golden fixtures (tests/golden/).
Everything else runs on CPU.
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd")
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X) and the built library")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # Build the CPU checker once (cheap; g++ only).
    from oracle import pyoracle

    pyoracle.build_oracle()
