"""bench.py's timed loop with consecutive steps round-robin over HIP streams (--streams): every
stream's outputs equal the one-stream run's, symbol for symbol, on the same batch, and equal the
transmitted symbols (noiseless frames)."""
import os
import sys

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    import bench as b

    b.PREWARM_MS = 20.0
    return b


@pytest.mark.parametrize("sf,frames", [(7, 512), (12, 16)])
def test_streams_match_one_stream(bench, sf, frames):
    dev = torch.device("cuda", 0)
    inputs = bench.make_input(sf, frames, 16, 777, dev, None)
    r1 = bench.run_config(sf, frames, 16, 6, 2, None, dev, inputs=inputs, streams=1)
    r3 = bench.run_config(sf, frames, 16, 7, 2, None, dev, inputs=inputs, streams=3)
    assert r1["streams"] == 1 and r3["streams"] == 3
    assert r1["symbols_ok"] and r3["symbols_ok"]
    assert torch.equal(r1["out"].symbols, r3["out"].symbols)
    assert torch.equal(r1["out"].sync, r3["out"].sync)
    assert torch.equal(r1["out"].cfo.view(torch.int32), r3["out"].cfo.view(torch.int32))
