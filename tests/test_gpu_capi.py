"""GPU: C-ABI contract beyond parity - error codes (the reference's -1 paths), stream
ordering, hipGraph capture, and the no-allocation rule (no_alloc_test.cpp)."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def amd():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import lora_phy_amd

    return lora_phy_amd


def test_batch_error_codes(amd):
    from lora_phy_amd import _capi

    lib = _capi.lib()
    plan = amd.DemodPlan(7)
    F, L = 4, 66 * 128
    iq = torch.zeros((F, L), dtype=torch.complex64, device="cuda")
    syms = torch.zeros((F, 64), dtype=torch.uint16, device="cuda")
    ws = torch.zeros(lib.lora_demod_workspace_bytes(plan._h, F, L), dtype=torch.uint8, device="cuda")
    out = _capi.DemodOutputs(syms.data_ptr(), 64, None, None, None, None)
    ok = lib.lora_demod_batch(plan._h, iq.data_ptr(), F, L, L, C.byref(out), ws.data_ptr(), ws.numel(), None)
    assert ok == 64
    # workspace too small / missing -> -ERANGE (reference: scratch too small returns 0)
    assert lib.lora_demod_batch(plan._h, iq.data_ptr(), F, L, L, C.byref(out), ws.data_ptr(), 16, None) \
        == _capi.LORA_ERANGE
    # output capacity too small -> -ERANGE (phy.cpp:190)
    small = _capi.DemodOutputs(syms.data_ptr(), 10, None, None, None, None)
    assert lib.lora_demod_batch(plan._h, iq.data_ptr(), F, L, L, C.byref(small), ws.data_ptr(), ws.numel(),
                                None) == _capi.LORA_ERANGE
    # null iq, stride < length -> -EINVAL
    assert lib.lora_demod_batch(plan._h, None, F, L, L, C.byref(out), ws.data_ptr(), ws.numel(), None) \
        == _capi.LORA_EINVAL
    assert lib.lora_demod_batch(plan._h, iq.data_ptr(), F, L, L - 1, C.byref(out), ws.data_ptr(), ws.numel(),
                                None) == _capi.LORA_EINVAL
    assert lib.lora_last_error().decode()
    # zero frames is a no-op that still reports symbols per frame
    assert lib.lora_demod_batch(plan._h, iq.data_ptr(), 0, L, L, C.byref(out), None, 0, None) == 64


def test_runs_on_the_callers_stream(amd):
    sf = 8
    syms = torch.randint(0, 256, (64, 20), dtype=torch.int32)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        iq = amd.modulate(syms.cuda(), sf)
        res = amd.DemodPlan(sf, dechirp=True).run(iq)
    s.synchronize()
    assert torch.equal(res.symbols.to(torch.int32).cpu(), syms)


def test_hip_graph_capture_and_replay(amd):
    """lora_demod_batch enqueues only kernels on the given stream (no allocation, no
    sync), so it can be captured into a HIP graph and replayed."""
    sf = 7
    syms = torch.randint(0, 128, (512, 64), dtype=torch.int32)
    iq = amd.modulate(syms.cuda(), sf)
    plan = amd.DemodPlan(sf, dechirp=True)
    out = plan.run(iq)
    torch.cuda.synchronize()
    out.symbols.zero_()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        plan.run(iq, out)  # warm the stream-side state before capture
    torch.cuda.current_stream().wait_stream(s)
    out.symbols.zero_()
    with torch.cuda.graph(g):
        plan.run(iq, out)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out.symbols.to(torch.int32).cpu(), syms)
    # new input in the same buffer -> replay demodulates it
    syms2 = torch.randint(0, 128, (512, 64), dtype=torch.int32)
    iq.copy_(amd.modulate(syms2.cuda(), sf))
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out.symbols.to(torch.int32).cpu(), syms2)


def test_no_device_allocation_per_call(amd):
    """no_alloc_test.cpp: the hot call allocates nothing (torch's allocator stats stay
    flat when outputs and workspace are reused)."""
    sf = 9
    syms = torch.randint(0, 512, (32, 30), dtype=torch.int32)
    iq = amd.modulate(syms.cuda(), sf)
    plan = amd.DemodPlan(sf, dechirp=True)
    out = plan.run(iq)
    torch.cuda.synchronize()
    before = torch.cuda.memory_stats()["allocation.all.allocated"]
    for _ in range(5):
        plan.run(iq, out)
    torch.cuda.synchronize()
    assert torch.cuda.memory_stats()["allocation.all.allocated"] == before
    assert torch.equal(out.symbols.to(torch.int32).cpu(), syms)


def test_wrapper_rejects_bad_tensors(amd):
    """The ctypes wrappers check what the C library cannot: a CPU, wrong-dtype,
    strided or short tensor raises instead of reaching a kernel as a raw pointer."""
    plan = amd.DemodPlan(7)
    F, L = 4, 20 * 128
    iq = torch.zeros((F, L), dtype=torch.complex64, device="cuda")
    with pytest.raises(TypeError):
        plan.run(iq.cpu())
    with pytest.raises(TypeError):
        plan.run(torch.zeros((F, 2 * L), dtype=torch.float32, device="cuda"))
    with pytest.raises(ValueError):
        plan.run(torch.zeros((L, F), dtype=torch.complex64, device="cuda").t())
    cfo = torch.zeros(F, dtype=torch.float32, device="cuda")
    toff = torch.zeros(F, dtype=torch.float32, device="cuda")
    with pytest.raises(TypeError):
        plan.estimate_offsets(iq, cfo.cpu(), toff)
    with pytest.raises(TypeError):
        plan.estimate_offsets(iq, cfo.double(), toff)
    with pytest.raises(ValueError):
        plan.estimate_offsets(iq, cfo[:2], toff)
    with pytest.raises(ValueError):
        amd.compensate_offsets(iq, 7, 1, cfo, toff[:1])
    with pytest.raises(TypeError):
        amd.compensate_offsets(iq, 7, 1, cfo.half(), toff)
    res = plan.run(iq)
    res.cfo = res.cfo[:1]
    with pytest.raises(ValueError):
        plan.run(iq, out=res)
    assert plan.estimate_offsets(iq, cfo, toff) == 20


def test_workspace_per_stream(amd):
    """Runs on two streams use two workspaces (no shared frame maxima / FrameParams)."""
    plan = amd.DemodPlan(7, dechirp=True)
    iq = amd.modulate(torch.randint(0, 128, (64, 64), device="cuda", dtype=torch.int32), 7)
    ref = plan.run(iq).symbols.clone()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        r1 = plan.run(iq)
    with torch.cuda.stream(s2):
        r2 = plan.run(iq)
    torch.cuda.synchronize()
    assert len(plan._ws) >= 3
    assert torch.equal(r1.symbols, ref) and torch.equal(r2.symbols, ref)


def test_lora_demod_mtu_caps_symbols_per_frame(amd):
    syms = torch.randint(0, 128, (4, 30), device="cuda", dtype=torch.int32)
    iq = amd.modulate(syms, 7)
    d = amd.LoRaDemod(7, mtu=20)
    out = d.work(iq)
    assert out.shape == (4, 20)
    assert torch.equal(out.to(torch.int32), syms[:, :20])
    assert d.last.symbols.shape == (4, 30)
