"""Experiment: does replaying lora_demod_batch from a HIP graph (torch.cuda.CUDAGraph
stream capture) shorten the SF7 bench step?  Prints eager vs graph ms/step."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd"))
import lora_phy_amd as amd  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
g = torch.Generator().manual_seed(1)
syms = torch.randint(0, 128, (15625, 64), generator=g, dtype=torch.int32)
iq = amd.modulate(syms.to(dev), 7)
plan = amd.DemodPlan(7, 1, 125000, "none", dechirp=True)
out = plan.run(iq)
torch.cuda.synchronize()
steps = 50


def timeit(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


eager = timeit(lambda: plan.run(iq, out))
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    plan.run(iq, out)
torch.cuda.current_stream().wait_stream(s)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    plan.run(iq, out)
graphed = timeit(graph.replay)
ok = torch.equal(out.symbols.to(torch.int32).cpu(), syms)
print(f"eager {eager:.4f} ms/step   graph {graphed:.4f} ms/step   symbols_ok {ok}")
