"""bench.py forms N ranks by itself (no torchrun, no RCCL): the multi-GPU launch path
that the driver's N = 2/4/8 runs use, rehearsed on CPU with gloo and --plumbing (the
ranks form, report their device ordinals and the max/sum reductions, and touch no GPU)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True,
                       text=True, timeout=120, env=e, cwd=REPO)
    return p


@pytest.mark.parametrize("n", [1, 2, 4])
def test_bench_forms_n_ranks(n):
    p = _run(["--gpus", str(n), "--plumbing"])
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    # stdout is exactly one JSON line, from rank 0 only (gloo's connection reports go to
    # stderr: the driver parses the job's stdout)
    assert len(lines) == 1 and lines[0].startswith("{"), p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert [r["rank"] for r in d["ranks"]] == list(range(n))
    assert [r["device"] for r in d["ranks"]] == list(range(n))  # one device per rank
    assert len({r["pid"] for r in d["ranks"]}) == n  # one process per rank
    assert d["max_seconds"] == pytest.approx(0.001 * n)  # max over ranks
    assert d["units"] == pytest.approx(1000.0 * n)  # sum over ranks


def test_bench_rejects_world_mismatch():
    p = _run(["--gpus", "2", "--plumbing"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr
