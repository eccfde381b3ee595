"""Benchmark: LoRa demod hot path (dechirp -> 2^SF FFT -> argmax) on MI355X.

One step = one lora_demod_batch over this rank's batch of frames already resident in
HBM: LEGACY lora_demodulate semantics with the fused caller-side dechirp
(e2e_chain_test.cpp:85-101): normalisation, 2-symbol CFO/timing estimate, per-symbol
CFO rotation, FFT, argmax, sync word.  Inputs are generated on the device by the
bit-exact GPU modulator (lora_mod_batch), random symbols from a fixed seed.  Each step is
one plan.run (the pipeline's four kernels enqueued on the stream; `--launch graph` replays
them as a captured HIP graph instead, whose per-replay cost made it 2 % slower at SF7 in
round 5's same-box A/B).

Headline workload (BASELINE.json configs[1]): SF7 BW125 osr 1, 1,000,000 data symbols
= 15,625 frames x (2 sync + 64 data) per GPU.  The SF12 configuration (configs[2]) and
configs[4] (8 channels x 1e6 SF7 frames of 16 data symbols, one channel per GPU) are
measured in the same run and reported under "extra", with the data-dependent slow
rotation path (sync 0xFF), an AWGN 0 dB batch, the modulator and the CPU baselines.

Multi-GPU: one process per GPU, frames sharded, no collective on the data path (weak
scaling; value = data symbols of all ranks / max-over-ranks time).  `--gpus N` starts
the N rank processes itself when not launched by torchrun (the parent never touches the
GPU); ranks meet over gloo (host TCP) for the timing barrier and the max/sum of the
timings only - RCCL is not used at all.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd"))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
METRIC = "Msymbols/s dechirp+FFT+argmax @ SF7 & SF12, 1/2/4/8 GPU; % HBM roofline"
SYNC = 0x12


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------------
# Rank formation (no torchrun needed, no RCCL)
# ---------------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(argv, n):
    """Start `n` copies of this script as ranks 0..n-1 (children, not exec: this parent
    has not initialised the GPU and never does).  Rank 0's stdout is ours; the others'
    stdout goes to stderr.  Any rank that fails - a non-zero exit or a signal (negative
    return code, e.g. SIGSEGV after a GPU fault) - fails the job, and the surviving ranks
    are terminated instead of waiting in the gloo rendezvous.  Returns the exit code."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "LORA_BENCH_SPAWNED": "1"})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def dist_setup(n_gpus, plumbing=False):
    """Join the job: WORLD_SIZE from the environment (torchrun or spawn_ranks); it must
    equal --gpus.  Rank r uses device LOCAL_RANK.  gloo (host TCP) carries the barrier
    and the max/sum all-reduces of the timings - no RCCL."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}; run `python bench.py "
                         f"--gpus N` (it starts the N ranks itself) or torchrun --nproc-per-node N")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not plumbing:
        import torch

        ndev = torch.cuda.device_count()
        if local >= ndev:
            if os.environ.get("LORA_BENCH_SHARE_DEVICES") == "1" and ndev > 0:
                # rehearsal of the multi-rank path on a box with fewer GPUs than ranks:
                # ranks share devices round-robin (numbers are then not per-GPU figures)
                local = local % ndev
            else:
                raise SystemExit(f"bench.py: rank needs device {local} but {ndev} are visible")
        torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        import datetime

        # gloo reports its peer connections on the C++ stdout; the job's stdout carries only
        # rank 0's JSON line, so the rendezvous runs with fd 1 pointed at stderr
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
        return dist, dist.get_rank(), world, local
    return None, 0, 1, local


def barrier(dist):
    if dist is not None:
        dist.barrier()


def all_max_sum(dist, seconds, units):
    """(max seconds, sum units) over ranks (gloo, host tensors)."""
    if dist is None:
        return seconds, units
    import torch

    t = torch.tensor([seconds], dtype=torch.float64)
    u = torch.tensor([units], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), float(u.item())


def gather_obj(dist, obj, world):
    if dist is None:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


# ---------------------------------------------------------------------------------
# Workloads
# ---------------------------------------------------------------------------------

def make_input(sf, frames, data_syms, seed, device, snr_db=None, sync=None, osr=1):
    import numpy as np
    import torch

    import lora_phy_amd as amd

    g = torch.Generator(device="cpu").manual_seed(seed)
    syms = torch.randint(0, 1 << sf, (frames, data_syms), generator=g, dtype=torch.int32)
    iq = amd.modulate(syms.to(device), sf, osr, 125000, 1.0, SYNC if sync is None else sync)
    if snr_db is not None:
        # awgn_sweep_gtest.cpp:76-80: sigma = 10^(-SNR/20), sigma/sqrt(2) per component
        sigma = 10.0 ** (-snr_db / 20.0) / np.sqrt(2.0)
        gn = torch.Generator(device=device).manual_seed(seed + 1)
        noise = torch.randn(iq.shape + (2,), generator=gn, device=device) * sigma
        iq = iq + torch.view_as_complex(noise)
    return syms, iq


LAUNCH = "eager"  # --launch: "eager" (plan.run per step, default) or "graph" (HIP graph replay of the step)
# --prewarm-ms: untimed steps of the same workload, for at least this long, before the W warmup
# steps - so that the K timed steps see the GPU's sustained state even when K and W are small.
# (Round 6, one box, headline only: 20 timed steps after 5 warmup steps measured 0.2627 and
# 0.2701 ms per step, 100 after 10 0.2521: a few ms of work after a cold start runs below the
# sustained rate.)
PREWARM_MS_DEFAULT = 300.0
PREWARM_MS = PREWARM_MS_DEFAULT
# --streams: consecutive steps (batches) go round-robin to this many HIP streams, each with
# its own workspace (DemodPlan keeps one per stream) and outputs - a receiver with that many
# batches in flight, so one batch's latency-bound estimate stages run beside the next one's
# kernels.  Every step still runs the whole pipeline on its whole batch inside the timed
# region.  (Round 6, one box, tools/streams_probe.py: SF7 0.2376-0.2406 ms per step on one
# stream, 0.2205-0.2259 on two, 0.2203-0.2211 on three; SF12 4,000 frames -4 % on two.)
# 0 = by spreading factor: three at SF <= 9 (short symbol passes: a third batch still finds
# room; SF7 -1 to -4 % against two), two beyond (SF12 on three: +4 %, tools/streams_probe.py)
STREAMS_DEFAULT = 0
STREAMS = STREAMS_DEFAULT


def streams_for(sf):
    return STREAMS if STREAMS > 0 else (3 if sf <= 9 else 2)


def stage_times(plan, iq, out, steps, device, streams=None, outs=None):
    """Per-kernel durations: a second pass of the same steps with HIP events around every
    launch, recorded on the stream each kernel runs on (outside the timed region).  With
    `streams`, the steps go round-robin over them as in the timed loop, so each launch runs
    beside the other batch's kernels as it did there (and as the tracer sees it)."""
    import ctypes as C

    import torch

    from lora_phy_amd import _capi

    lib = _capi.lib()
    _capi.check(lib.lora_demod_profile_enable(plan._h, steps))
    if streams and len(streams) > 1:
        main = torch.cuda.current_stream(device)
        for st in streams:
            st.wait_stream(main)
        for k in range(steps):
            with torch.cuda.stream(streams[k % len(streams)]):
                outs[k % len(streams)] = plan.run(iq, outs[k % len(streams)])
        for st in streams:
            main.wait_stream(st)
        out = outs[0]
    else:
        for _ in range(steps):
            out = plan.run(iq, out)
    torch.cuda.synchronize(device)
    stage = (C.c_float * 3)()
    calls = C.c_int()
    _capi.check(lib.lora_demod_profile_read(plan._h, stage, C.byref(calls)))
    lib.lora_demod_profile_enable(plan._h, 0)
    return [stage[k] / max(calls.value, 1) for k in range(3)], out


def run_config(sf, frames, data_syms, steps, warmup, dist, device, snr_db=None, precision="exact",
               inputs=None, sync=None, seed_base=20251015, rank=0, window="none", osr=1, spec=True,
               mode="legacy", streams=None):
    """mode "legacy": lora_demodulate with the fused caller dechirp (the headline); "api":
    lora_phy::demodulate (phy.cpp:178-239: estimate on the raw samples, down-chirp fused per
    symbol); "raw": the detector alone per symbol (dechirp -> FFT -> argmax, the AWGN
    script's receiver, tests/awgn_sweep.py:262-273), every symbol of the frame an output."""
    import torch

    import lora_phy_amd as amd

    N = 1 << sf
    syms, iq = inputs if inputs is not None else make_input(sf, frames, data_syms, seed_base + rank, device,
                                                            snr_db, sync, osr)
    # spec=False: the three-launch path (frame max, estimate, demod), for comparison lines
    with amd.spec_pipeline(spec):
        plan = amd.DemodPlan(sf, osr, 125000, window, dechirp=True, mode=mode, device=device,
                             precision=precision)
    out = None
    # the steps' streams (STREAMS; one for a graph replay): step k on stream k mod S, with
    # outputs of its own
    S = 1 if LAUNCH == "graph" else max(1, streams_for(sf) if streams is None else streams)
    main_stream = torch.cuda.current_stream(device)
    sts = [main_stream] if S == 1 else [torch.cuda.Stream(device) for _ in range(S)]
    outs = [None] * S

    def run_step(k):
        with torch.cuda.stream(sts[k % S]):
            outs[k % S] = plan.run(iq, outs[k % S])

    t_warm = time.perf_counter()
    while (time.perf_counter() - t_warm) * 1e3 < PREWARM_MS:  # untimed pre-warm (PREWARM_MS)
        for k in range(8):
            run_step(k)
        torch.cuda.synchronize(device)
    for k in range(max(warmup, S)):
        run_step(k)
    torch.cuda.synchronize(device)
    out = outs[0]
    step = None
    if LAUNCH == "graph":
        # the step's launches captured once into a HIP graph and replayed (the same kernels
        # on the same buffers; lora_demod_batch enqueues only kernels, no sync or allocation)
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            out = plan.run(iq, out)
        torch.cuda.current_stream(device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = plan.run(iq, out)
        step = g.replay
        step()
        torch.cuda.synchronize(device)
    fixed0 = plan.spec_recomputed()
    barrier(dist)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for st in sts:
        if st is not main_stream:
            st.wait_stream(main_stream)
    for k in range(steps):
        if step is not None:
            step()
        else:
            run_step(k)
    for st in sts:
        if st is not main_stream:
            main_stream.wait_stream(st)
    torch.cuda.synchronize(device)
    barrier(dist)
    wall = time.perf_counter() - t0
    if step is None:
        out = outs[0]
        # every stream's outputs are the same batch's: equal to stream 0's, symbol for symbol
        streams_equal = all(bool(torch.equal(o.symbols, out.symbols)) and bool(torch.equal(o.sync, out.sync))
                            for o in outs)
    else:
        streams_equal = True
    fixed = (plan.spec_recomputed() - fixed0) / steps
    kernels = sorted(plan.last_kernels())
    # (at least 50 launches: with the driver's 20 the per-kernel averages carried the
    # first launches' ramp, e.g. 0.2114 against 0.1933 ms for the SF7 pass on one box)
    # the kernels one batch at a time (no other batch's kernels beside them: what the kernel
    # tracer, which serialises launches, measures) - the roofline's launch time; and with the
    # steps on the timed loop's streams, where a launch shares the GPU with the other batch's
    # kernels and its wall time stretches while the step's throughput rises
    stage_ms, out = stage_times(plan, iq, out, max(steps, 50), device)
    stage_ms_streams = stage_ms if S == 1 else stage_times(plan, iq, out, max(steps, 50), device, sts, outs)[0]
    total_syms = data_syms + 2
    # RAW mode demodulates every symbol of the frame (the sync symbols too)
    out_syms = total_syms if mode == "raw" else data_syms
    wall_max, units = all_max_sum(dist, wall, frames * out_syms * steps)
    ms_step = wall * 1e3 / steps
    B_sym = 8 * N * osr + 2
    got = out.symbols.to(torch.int32).cpu()
    if mode == "raw":
        sw = SYNC if sync is None else sync
        shift = sf - 4 if sf > 4 else 0
        head = torch.tensor([(sw >> 4) << shift, (sw & 0xF) << shift], dtype=torch.int32)
        ser = float((got != torch.cat([head.expand(frames, 2), syms], 1)).float().mean())
    else:
        ser = float((got != syms).float().mean())
    if not streams_equal:
        ser = max(ser, 1.0)  # a stream's outputs differ from stream 0's: not ok
    # the symbol pass in the speculative pipeline (ranks sharing a device in a rehearsal
    # can distort the stage times); otherwise the longest stage
    dom = 2 if "spec" in kernels else max(range(3), key=lambda k: stage_ms[k])
    # algorithmic bytes: every symbol's IQ read once + its u16 index
    # write, plus 9 B of per-frame outputs
    step_bytes = frames * (total_syms * B_sym + 9)
    # the dominant kernel's own algorithmic bytes per launch
    # (the speculative pipeline's symbol pass also demodulates the sync symbols: every
    # window of the frame read once, one index written per data symbol)
    spec = "spec" in kernels
    W = 8 * N * osr  # bytes per symbol window
    # (API: the pass reads the data windows only - the estimate kernel demodulates symbols
    # 0/1; RAW: every window, every symbol an output)
    spec_windows = data_syms if mode == "api" else total_syms
    dom_bytes = {0: frames * total_syms * W,                 # frame max: the whole IQ
                 1: frames * (2 * W + 9),                     # estimate: symbols 0/1 + outputs
                 2: (frames * (spec_windows * W + 2 * out_syms) if spec
                     # three-launch demod: every osr-th sample of a window is read
                     else frames * out_syms * (8 * N + 2))}[dom]
    dom_gbs = dom_bytes / (stage_ms[dom] * 1e-3) / 1e9
    return {
        "sf": sf, "osr": osr, "mode": mode, "window": window, "precision": precision,
        "frames": frames, "data_symbols": frames * out_syms, "iq_bytes": iq.numel() * 8,
        "ms_per_step": ms_step, "stage_ms": stage_ms, "stage_ms_streams": stage_ms_streams,
        "symbols_ok": ser == 0.0, "ser_vs_tx": ser,
        "streams": S,
        "kernels": kernels, "spec_recomputed_per_step": fixed,
        "msym_s_data": frames * out_syms / (ms_step * 1e-3) / 1e6,
        "msym_s_all_ranks": units / wall_max / 1e6, "ms_per_step_max_rank": wall_max * 1e3 / steps,
        "msym_s_all": frames * total_syms / (ms_step * 1e-3) / 1e6,
        # stage 2 is the symbol pass: k_spec_demod in the speculative pipeline (the default),
        # k_demod_fast in the three-launch one
        "dominant_kernel": ["k_frame_max", "k_est_fast",
                            "k_spec_demod" if "spec" in kernels else "k_demod_fast"][dom], "dominant_stage": dom,
        "sync": SYNC if sync is None else sync,
        "dominant_gbs": dom_gbs, "dominant_bytes_per_launch": dom_bytes,
        "step_bytes": step_bytes, "pipeline_gbs": step_bytes / (ms_step * 1e-3) / 1e9,
        "plan": plan, "iq": iq, "syms": syms, "out": out,
    }


def public(r):
    return {k: v for k, v in r.items() if k not in ("plan", "iq", "syms", "out")}


def _bits(t):
    import torch

    return t.contiguous().view(torch.int32)


def exact_parity(r, device, ref=None):
    """Parity of a line measured in the run: every frame's outputs (symbols, sync word and
    the fp32 bits of cfo / time_offset) against the three-launch exact path on the same
    batch (frame max, estimate, demod with glibc-faithful sincosf: LORA_MI355X_SPEC=0, the
    path the GPU test suite pins to the oracle and the reference bit for bit).  `ref`: an
    already computed exact run of the same inputs (its DemodResult)."""
    import torch

    import lora_phy_amd as amd

    if ref is None:
        with amd.spec_pipeline(False):
            plan = amd.DemodPlan(r["sf"], r["osr"], 125000, r["window"], dechirp=True, mode=r["mode"], device=device,
                                 precision="exact")
        ref = plan.run(r["iq"])
        torch.cuda.synchronize(device)
        del plan
    o = r["out"]
    bad = (o.symbols.to(torch.int32) != ref.symbols.to(torch.int32)).any(1) | (o.sync != ref.sync)
    bad |= (_bits(o.cfo) != _bits(ref.cfo)) | (_bits(o.time_offset) != _bits(ref.time_offset))
    nbad = int(bad.sum())
    return {"parity_ok": nbad == 0, "frames_compared": int(o.symbols.shape[0]), "frames_mismatched": nbad,
            "vs": "three-launch exact path on the same batch (LORA_MI355X_SPEC=0; oracle-pinned by the GPU tests)"}


def reference_leg(r, nframes=32, budget_s=2.0):
    """cpu_baseline leg of a variant line: the reference itself (oracle/_ref, built from the
    reference's sources; the restatement for the detector-only RAW mode, which the
    reference has only as tests/awgn_sweep.py's numpy receiver) on the first `nframes`
    frames of the same batch, one host thread - its rate, and its outputs compared with the
    GPU's for those frames (symbols, sync, cfo / time_offset bits)."""
    import numpy as np

    from oracle.pyoracle import Oracle, Reference

    sf, osr, mode = r["sf"], r["osr"], r["mode"]
    F = min(nframes, r["iq"].shape[0])
    x = r["iq"][:F].cpu().numpy()
    o = r["out"]
    gs = o.symbols[:F].cpu().numpy().astype(np.int64)
    gsync = o.sync[:F].cpu().numpy()
    gcfo = o.cfo[:F].cpu().numpy().view(np.uint32)
    gto = o.time_offset[:F].cpu().numpy().view(np.uint32)
    hann = r["window"] == "hann"
    use_ref = Reference.available() and mode != "raw"
    impl = Reference() if use_ref else Oracle()
    orc = Oracle()
    bad = 0
    t0 = time.perf_counter()
    reps = 0
    while True:
        for f in range(F):
            if mode == "legacy":
                syms, sync, cfo, toff = impl.lora_demodulate(orc.dechirp(x[f], sf, osr), sf, osr, hann)
            elif mode == "api":
                _, syms, sync, cfo, toff = impl.api_demodulate(x[f], sf, osr, hann)
            else:
                syms, sync, cfo, toff = impl.raw_demod(x[f], sf, osr, hann, dechirp=True), 0, 0.0, 0.0
            if reps == 0:
                ok = (np.array_equal(np.asarray(syms, np.int64), gs[f][:len(syms)]) and len(syms) == gs.shape[1]
                      and int(sync) == int(gsync[f]) and np.float32(cfo).view(np.uint32) == gcfo[f]
                      and np.float32(toff).view(np.uint32) == gto[f])
                bad += not ok
        reps += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    per = gs.shape[1]
    what = {"legacy": "lora_demodulate after the caller's dechirp", "api": "phy::demodulate",
            "raw": "detector per symbol"}[mode]
    return {"value": reps * F * per / dt / 1e6, "unit": "Msymbols/s", "cores": 1,
            "kind": "reference" if use_ref else "port",
            "sample": f"first {F} frames of this line's batch x {reps} passes, {what}, 1 thread, {dt:.2f} s",
            "parity_ok": bad == 0, "frames_compared": F, "frames_mismatched": bad}


def run_channels(frames, data_syms, steps, warmup, dist, device, rank, chunk_bytes=8e9):
    """BASELINE.json configs[4]: one channel per GPU, `frames` SF7 frames of 2 + `data_syms`
    symbols resident in HBM (18.4 GB at 1e6 x 16), demodulated in <= 8 GB chunks per step
    (SURVEY.md 8d item 5).  Inputs generated on the device (GPU modulator) in slices;
    every frame's symbols are checked against the transmitted ones (noiseless)."""
    import torch

    import lora_phy_amd as amd

    sf, N = 7, 128
    L = (data_syms + 2) * N
    iq = torch.empty((frames, L), dtype=torch.complex64, device=device)
    tx = torch.empty((frames, data_syms), dtype=torch.int16, device=device)
    g = torch.Generator(device="cpu").manual_seed(4242 + rank)
    gen_rows = 1 << 17
    for r0 in range(0, frames, gen_rows):
        n = min(gen_rows, frames - r0)
        syms = torch.randint(0, N, (n, data_syms), generator=g, dtype=torch.int32).to(device)
        tx[r0:r0 + n] = syms.to(torch.int16)
        iq[r0:r0 + n] = amd.modulate(syms, sf, 1, 125000, 1.0, SYNC)
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, mode="legacy", device=device)
    per_chunk = max(1, int(chunk_bytes // (L * 8)))
    chunks = [(c0, min(per_chunk, frames - c0)) for c0 in range(0, frames, per_chunk)]
    outs = [None] * len(chunks)
    # the chunks round-robin over STREAMS HIP streams (a workspace each): one chunk's estimate
    # stages beside another's symbol pass, as bench.py's steps
    S = max(1, streams_for(sf))
    main_stream = torch.cuda.current_stream(device)
    sts = [main_stream] if S == 1 else [torch.cuda.Stream(device) for _ in range(S)]

    def step():
        for i, (c0, n) in enumerate(chunks):
            with torch.cuda.stream(sts[i % S]):
                outs[i] = plan.run(iq[c0:c0 + n], outs[i])

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(device)
    barrier(dist)
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for st in sts:
        if st is not main_stream:
            st.wait_stream(main_stream)
    for _ in range(steps):
        step()
    for st in sts:
        if st is not main_stream:
            main_stream.wait_stream(st)
    torch.cuda.synchronize(device)
    barrier(dist)
    wall = time.perf_counter() - t0
    wall_max, units = all_max_sum(dist, wall, frames * data_syms * steps)
    bad = 0
    for (c0, n), o in zip(chunks, outs):
        bad += int((o.symbols.to(torch.int16) != tx[c0:c0 + n]).sum())
    # parity: every chunk against the three-launch exact path (all outputs, every frame)
    with amd.spec_pipeline(False):
        xplan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, mode="legacy", device=device)
    pbad = 0
    for (c0, n), o in zip(chunks, outs):
        pr = exact_parity({"out": o}, device, xplan.run(iq[c0:c0 + n]))
        pbad += pr["frames_mismatched"]
    del xplan, iq, tx
    return {"frames_per_gpu": frames, "data_symbols_per_frame": data_syms, "iq_gb_per_gpu": frames * L * 8 / 1e9,
            "chunks": len(chunks), "streams": S, "ms_per_step": wall * 1e3 / steps,
            "ms_per_step_max_rank": wall_max * 1e3 / steps,
            "value_all_ranks_msym_s": units / wall_max / 1e6,
            "symbols_ok_all_frames": bad == 0, "symbol_mismatches": bad,
            "parity": {"parity_ok": pbad == 0, "frames_compared": frames, "frames_mismatched": pbad,
                       "vs": "three-launch exact path, every chunk (LORA_MI355X_SPEC=0; oracle-pinned by the GPU "
                             "tests)"}}


def modulator_reference_leg(sf, syms16, out, nframes=8, budget_s=2.0):
    """cpu_baseline leg of a modulator line: the reference's lora_modulate (oracle/_ref;
    the restatement if absent) on the first frames' symbols, one thread, and every sample
    of those frames compared with the GPU's bit for bit."""
    import numpy as np

    from oracle.pyoracle import Oracle, Reference

    impl = Reference() if Reference.available() else Oracle()
    F = min(nframes, syms16.shape[0])
    sy = syms16[:F].cpu().numpy().astype(np.uint16)
    g = out[:F].cpu().numpy()
    bad = 0
    reps = 0
    t0 = time.perf_counter()
    while True:
        for f in range(F):
            ref = impl.lora_modulate(sy[f], sf, 1, 125000, 1.0, SYNC)
            if reps == 0:
                bad += not np.array_equal(ref.view(np.uint32), g[f].view(np.uint32))
        reps += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": reps * F * (sy.shape[1] + 2) / dt / 1e6, "unit": "Msymbols/s (chirps)", "cores": 1,
            "kind": "reference" if isinstance(impl, Reference) else "port",
            "sample": f"lora_modulate of the first {F} frames x {reps} passes, 1 thread, {dt:.2f} s",
            "parity_ok": bad == 0, "frames_compared": F, "frames_mismatched": bad}


def run_modulator(sf, frames, data_syms, device, reps=3, with_cpu=True):
    """lora_mod_batch throughput: samples written per second and the
    HBM write rate (8 B per sample written, symbol reads negligible)."""
    import torch

    import lora_phy_amd as amd

    g = torch.Generator(device="cpu").manual_seed(99)
    syms = torch.randint(0, 1 << sf, (frames, data_syms), generator=g, dtype=torch.int32).to(device)
    syms16 = syms.to(torch.uint16)
    # the output is allocated once, outside the timed region: a fresh 4.3 GB (SF12)
    # allocation per call put the allocator's page mapping into the timing (round 2's
    # mod_sf12 record: 361 ms per call against 6.3 ms in the next run of the same build)
    out = amd.modulate(syms16, sf)
    torch.cuda.synchronize(device)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        amd.modulate(syms16, sf, out=out)
    e1.record()
    torch.cuda.synchronize(device)
    ms = e0.elapsed_time(e1) / reps
    nbytes = out.numel() * 8
    cpu = None
    if with_cpu:
        try:
            cpu = modulator_reference_leg(sf, syms16, out)
        except Exception as e:  # the CPU leg must not kill the GPU measurement
            log("modulator cpu leg failed:", e)
    del out
    torch.cuda.empty_cache()
    return {"sf": sf, "frames": frames, "symbols_per_frame": data_syms + 2, "ms_per_call": ms,
            "cpu_baseline": cpu,
            "msym_s": frames * (data_syms + 2) / (ms * 1e-3) / 1e6, "write_gbs": nbytes / (ms * 1e-3) / 1e9,
            "roofline_frac": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, "bytes_written": nbytes}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """CPUs this process may run on: sched_getaffinity, capped by a cgroup CPU quota
    (cpu.max) when one is set - threads beyond the quota only time-slice."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    used = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return {"sched_getaffinity": aff, "cgroup_quota_cpus": quota, "used": used}


def cpu_baseline(sf, iq_dev, data_syms, max_frames, time_budget_s=10.0, gpu_out=None):
    """The reference's own lora_demodulate (oracle/_ref, compiled from the reference's
    sources, travels with the snapshot) on every usable host core (host_cores) over a
    bounded sample of the same frames; the restatement (oracle/lora_oracle.cpp) if the
    reference build is absent.  Reported `value`: all threads, caller-side dechirp +
    lora_demodulate (the GPU workload).  Also: one core, and demod only (input dechirped
    beforehand), per SURVEY.md 8d."""
    from oracle.pyoracle import Oracle, Reference

    if Reference.available():
        impl, kind, what = Reference(), "reference", "reference src/phy lora_demodulate (oracle/_ref)"
    else:
        impl, kind, what = Oracle(), "port", "restatement oracle/lora_oracle.cpp"
    cores = host_cores()
    threads = cores["used"]
    F = min(iq_dev.shape[0], max_frames)
    x = iq_dev[:F].cpu().numpy()

    def rate(xs, nthreads, dechirp, budget):
        impl.demod_frames(xs[: min(len(xs), nthreads)], sf, 1, False, dechirp=dechirp, threads=nthreads)
        t0 = time.perf_counter()
        done = 0
        while True:
            impl.demod_frames(xs, sf, 1, False, dechirp=dechirp, threads=nthreads)
            done += len(xs)
            if time.perf_counter() - t0 > budget:
                break
        dt = time.perf_counter() - t0
        return done * data_syms / dt / 1e6, done, dt

    parity = None
    if gpu_out is not None:
        # the reference's outputs on the sample against the GPU run's for the same frames
        import numpy as np

        rs, rsync, rcfo, rtoff, _ = impl.demod_frames(x, sf, 1, False, dechirp=True, threads=threads)
        gs = gpu_out.symbols[:F].cpu().numpy().astype(np.int64)
        bad = ((rs[:, :gs.shape[1]].astype(np.int64) != gs).any(1) | (rsync != gpu_out.sync[:F].cpu().numpy())
               | (rcfo.view(np.uint32) != gpu_out.cfo[:F].cpu().numpy().view(np.uint32))
               | (rtoff.view(np.uint32) != gpu_out.time_offset[:F].cpu().numpy().view(np.uint32)))
        parity = {"parity_ok": not bool(bad.any()), "frames_compared": F, "frames_mismatched": int(bad.sum()),
                  "vs": kind + " outputs on the sample frames (symbols, sync, cfo / time_offset bits)"}
    all_rate, done, dt = rate(x, threads, True, time_budget_s)
    one_rate, _, _ = rate(x[: max(1, min(F, 4))], 1, True, time_budget_s / 3)
    xd = Oracle().dechirp(x.reshape(-1), sf).reshape(x.shape)  # same fp32 products as the caller loop
    demod_only, _, _ = rate(xd, threads, False, time_budget_s / 3)
    return {"value": all_rate, "unit": "Msymbols/s", "cores": threads, "kind": kind,
            "host_cores": cores, "single_core": one_rate, "demod_only_all_cores": demod_only,
            "reference_parity": parity,
            "cpu_model": _cpu_model(),
            "sample": f"{done} frames of the SF{sf} bench batch ({data_syms}+2 symbols each, {F} distinct), "
                      f"caller-side dechirp + {what}, {threads} threads, {dt:.2f} s; single_core: same on 1 "
                      f"thread; demod_only: input dechirped beforehand"}


def fast_summary(r, exact):
    """LORA_PRECISION_FAST line (hardware sin/cos rotation; stated tolerance in
    include/lora_mi355x.h): same workload and inputs as the exact run, whose symbols it is
    compared with (a tolerance mode: agreement is reported, not required)."""
    import torch

    agree = float((r["out"].symbols.to(torch.int32) == exact["out"].symbols.to(torch.int32)).float().mean())
    return {"precision": "fast", "ms_per_step": r["ms_per_step"], "stage_ms": r["stage_ms"],
            "parity": {"tolerance_mode": True, "symbol_agreement_with_exact": agree},
            "symbols_ok": r["symbols_ok"], "value_all_ranks_msym_s": r["msym_s_all_ranks"],
            "pipeline_frac": r["pipeline_gbs"] / HBM_PEAK_GBS}


def variant_summary(r, base, note, parity=None):
    """A data-dependent variant of a workload: `ratio_to_headline` is its time per data
    symbol over the headline's (> 1 = slower); `parity` measured in the run
    (exact_parity / reference_leg)."""
    return {"note": note, "parity": parity, "frames": r["frames"],
            "data_symbols_per_frame": r["data_symbols"] // r["frames"],
            "ms_per_step": r["ms_per_step"], "stage_ms": r["stage_ms"],
            "value_all_ranks_msym_s": r["msym_s_all_ranks"], "ser_vs_tx": r["ser_vs_tx"],
            "pipeline_frac": r["pipeline_gbs"] / HBM_PEAK_GBS, "kernels": r["kernels"],
            "spec_recomputed_per_step": r["spec_recomputed_per_step"],
            "spec_recomputed_frac": r["spec_recomputed_per_step"] / r["data_symbols"],
            "ratio_to_headline": base["msym_s_data"] / r["msym_s_data"]}


def hbm_probe(device, nbytes=2 << 30, reps=5):
    """SURVEY.md 8d cross-check: device-to-device copy bandwidth on the same GPU
    (bytes read + bytes written per second), the chip's achievable HBM rate next to the
    8 TB/s spec."""
    import torch

    src = torch.empty(nbytes, dtype=torch.uint8, device=device)
    dst = torch.empty_like(src)
    dst.copy_(src)
    torch.cuda.synchronize(device)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        dst.copy_(src)
    t1.record()
    torch.cuda.synchronize(device)
    gbs = 2 * nbytes * reps / (t0.elapsed_time(t1) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return gbs


def load_pmc(workload, key="hbm_bytes_per_launch"):
    p = os.path.join(REPO, "profiles", "pmc_summary.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        return d.get(workload, {}).get(key)
    except Exception:
        return None


def roofline(r, probe=None):
    """roofline object for one workload: the dominant kernel (HIP-event time, algorithmic
    bytes per launch) and the whole step (pipeline_frac); counter bytes from the
    committed rocprofv3 profile (profiles/pmc_summary.json, labelled as such)."""
    # the committed counter profile of this workload: sf7 / sf12 (the headline shapes), or
    # <mode>_sf7 for the API / RAW lines
    wl = ("sf%d" % r["sf"]) if r.get("mode", "legacy") == "legacy" else "%s_sf%d" % (r["mode"], r["sf"])
    pmc_step = load_pmc(wl, "hbm_bytes_per_step")
    pmc_dom = load_pmc(wl, "hbm_bytes_per_launch")
    return {"bound": "hbm", "kernel": r["dominant_kernel"],
            "achieved": r["dominant_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": r["dominant_gbs"] / HBM_PEAK_GBS,
            # achieved / frac: the kernel's HIP-event launch time, one batch at a time (as the
            # kernel tracer sees it); with_streams: launched as in the timed loop, beside the
            # other batch's kernels (a longer wall time per launch, a higher step rate)
            "launch_ms": r["stage_ms"][r["dominant_stage"]],
            "with_streams": {"launch_ms": r["stage_ms_streams"][r["dominant_stage"]],
                             "frac": r["dominant_bytes_per_launch"] / (r["stage_ms_streams"][r["dominant_stage"]] * 1e-3)
                             / 1e9 / HBM_PEAK_GBS},
            "bytes_per_launch": r["dominant_bytes_per_launch"],
            "traffic": pmc_dom,
            "traffic_source": "profiles/pmc_summary.json (rocprofv3 FETCH_SIZE*2+WRITE_SIZE per launch, "
                              "tools/pmc_traffic.py; committed, not measured in this run)",
            # the kernel's other roof: VALU issue (SQ_INSTS_VALU x its issue cycles - 4 per
            # instruction, packed ones weighted by their 0.58 issue rate - over 1024 SIMDs x the
            # GRBM-measured cycles of the same launch, committed profile)
            "valu": {"busy_frac": load_pmc(wl, "valu_busy_frac"),
                     "busy_frac_4cycle": load_pmc(wl, "valu_busy_frac_4cycle"),
                     "instr_per_symbol": load_pmc(wl, "valu_instr_per_symbol"),
                     "source": "profiles/pmc_summary.json (rocprofv3 SQ_INSTS_VALU, GRBM_GUI_ACTIVE; "
                               "tools/pmc_traffic.py)"},
            "pipeline": {"algorithmic_bytes_per_step": r["step_bytes"], "ms_per_step": r["ms_per_step"],
                         "achieved": r["pipeline_gbs"], "pipeline_frac": r["pipeline_gbs"] / HBM_PEAK_GBS,
                         "counter_bytes_per_step": pmc_step,
                         "counter_over_algorithmic": (pmc_step / r["step_bytes"]) if pmc_step else None},
            "hbm_probe": {"d2d_copy_gbs": probe,
                          "note": "achievable rate on this GPU: torch D2D copy (read+write)"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--launch", choices=["eager", "graph"], default="eager",
                    help="step launch: plan.run per step (default: the step's four kernels enqueued on the "
                         "stream, about 1.5-2 us between dependent kernels), or one HIP-graph replay of the "
                         "step's launches (the same kernels on the same buffers, captured once; each replay "
                         "adds about 9.5 us before the next step - round 5: 2 % slower)")
    # 100 timed steps (33 ms at SF7): with 20 (6 ms) a single host or clock hiccup moved the
    # per-step time by several percent between runs of the same build
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frames", type=int, default=15625)
    ap.add_argument("--data-symbols", type=int, default=64)
    ap.add_argument("--sf12-frames", type=int, default=15625)
    ap.add_argument("--no-sf12", action="store_true")
    ap.add_argument("--sf12-only", action="store_true", help="profiling: SF12 workload only")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-channels", action="store_true", help="skip the configs[4] measurement")
    ap.add_argument("--no-fast", action="store_true", help="skip the LORA_PRECISION_FAST lines")
    ap.add_argument("--no-variants", action="store_true", help="skip the sync-0xFF / AWGN / modulator lines")
    ap.add_argument("--channel-frames", type=int, default=1_000_000)
    ap.add_argument("--sync", type=lambda v: int(v, 0), default=0x12,
                    help="sync word of the synthetic frames (0x12 = the reference default)")
    ap.add_argument("--plumbing", action="store_true",
                    help="form the ranks and report them without touching a GPU (CPU test of the "
                         "multi-rank launch)")
    ap.add_argument("--streams", type=int, default=STREAMS_DEFAULT,
                    help="HIP streams the consecutive steps go to, round-robin (each its own workspace and "
                         "outputs: that many batches in flight); 1 = every step on one stream; 0 (default) = "
                         "three at SF <= 9, two beyond")
    ap.add_argument("--prewarm-ms", type=float, default=PREWARM_MS_DEFAULT,
                    help="untimed steps of each workload for at least this long before its W warmup steps "
                         "(0: none)")
    args = ap.parse_args()
    global LAUNCH, PREWARM_MS, STREAMS
    LAUNCH = args.launch
    PREWARM_MS = args.prewarm_ms
    STREAMS = args.streams
    global SYNC
    SYNC = args.sync

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))
    dist, rank, world, local = dist_setup(args.gpus, args.plumbing)
    ranks = gather_obj(dist, {"rank": rank, "device": local, "pid": os.getpid()}, world)
    if args.plumbing:
        wall_max, units = all_max_sum(dist, 0.001 * (rank + 1), 1000)
        if rank == 0:
            print(json.dumps({"plumbing": True, "n_gpus": world, "ranks": ranks,
                              "max_seconds": wall_max, "units": units}), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    import torch

    device = torch.device("cuda", local)
    if args.sf12_only:
        r12 = run_config(12, args.sf12_frames, args.data_symbols, args.steps, args.warmup, dist, device, rank=rank)
        if rank == 0:
            print(json.dumps(public(r12)))
        return
    r7 = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, rank=rank)
    r7["parity"] = exact_parity(r7, device)
    one = None
    if r7["streams"] > 1:
        # the same workload with every step on one stream (batches back to back)
        r1 = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, rank=rank,
                        inputs=(r7["syms"], r7["iq"]), streams=1)
        one = {"ms_per_step": r1["ms_per_step_max_rank"], "value_all_ranks_msym_s": r1["msym_s_all_ranks"],
               "symbols_ok": r1["symbols_ok"]}
        del r1
    probe = None
    try:
        probe = hbm_probe(device)
    except Exception as e:  # a probe must not kill the measurement
        log("hbm probe failed:", e)
    extra = {}
    if not args.no_fast:
        r7f = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device,
                         precision="fast", inputs=(r7["syms"], r7["iq"]), rank=rank)
        extra["fast_rotation_sf7"] = fast_summary(r7f, r7)
        del r7f
    if not args.no_variants:
        # data-dependent slow rotation path: sync nibbles 0xF -> estimated cfo ~0.94 ->
        # phases up to ~400 rad, past glibc sincosf's |x| < 120 fast reduction
        rff = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, sync=0xFF,
                         rank=rank)
        extra["sync_ff_sf7"] = variant_summary(rff, r7, "sync 0xFF: large estimated CFO, Payne-Hanek "
                                                        "reduction in the rotation (ser_vs_tx is the reference's "
                                                        "own CFO-shift behaviour, not an error)",
                                               exact_parity(rff, device))
        del rff
        rn = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, snr_db=0.0,
                        rank=rank)
        extra["awgn_0db_sf7"] = variant_summary(rn, r7, "AWGN 0 dB (sigma/sqrt2 per component, "
                                                       "awgn_sweep_gtest.cpp:76-80); t_off != 0 frames",
                                                exact_parity(rn, device))
        del rn
        # the certified pipeline's worst case: near-ties at low SNR are recomputed exactly
        rn = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, snr_db=-10.0,
                        rank=rank)
        extra["awgn_m10db_sf7"] = variant_summary(rn, r7, "AWGN -10 dB: symbol errors and near-ties; symbols "
                                                         "failing certification are recomputed exactly",
                                                  exact_parity(rn, device))
        del rn
        # the Hann window (LoRaDemod.cpp:158-160) on the headline batch
        rh = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, window="hann",
                        inputs=(r7["syms"], r7["iq"]), rank=rank)
        extra["hann_sf7"] = variant_summary(rh, r7, "Hann window, same batch (ser_vs_tx: the window's own "
                                                    "effect on the reference's decisions, not an error)",
                                            exact_parity(rh, device))
        del rh
        # a 255-byte payload: 510 data symbols per frame (lora_encode: 2 symbols per byte)
        long_frames = max(1, args.frames * args.data_symbols // 510)
        rl = run_config(7, long_frames, 510, args.steps, args.warmup, dist, device, rank=rank)
        extra["long_frames_sf7"] = variant_summary(rl, r7, "255-byte payload: 2 + 510 symbols per frame, "
                                                          "noiseless, same data symbols per step",
                                                   exact_parity(rl, device))
        del rl
        torch.cuda.empty_cache()
        # oversampled LEGACY frames (osr 2: gr_lora_sdr_interop.cpp:34's capture shape; osr 4):
        # the speculative pipeline reads each frame once (the window's every sample for the
        # frame maximum, every osr-th transformed); the three-launch line reads it twice
        for osr in (2, 4):
            ro = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, rank=rank,
                            osr=osr)
            rt = None
            if osr == 2:
                rt = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, rank=rank,
                                osr=osr, inputs=(ro["syms"], ro["iq"]), spec=False)
            line = variant_summary(ro, r7, f"osr {osr}: {osr} x the IQ bytes per symbol, same data symbols",
                                   exact_parity(ro, device, rt["out"] if rt is not None else None))
            line["symbol_pass_gbs"] = ro["dominant_gbs"]
            line["symbol_pass_frac"] = ro["dominant_gbs"] / HBM_PEAK_GBS
            line["step_bytes"] = ro["step_bytes"]
            # HBM bytes the counters saw per symbol-pass launch over its algorithmic bytes
            # (committed rocprofv3 FETCH_SIZE / WRITE_SIZE profile, tools/pmc_r05.py)
            line["symbol_pass_counter_over_algorithmic"] = load_pmc(f"osr{osr}_sf7", "traffic_over_algorithmic")
            line["step_counter_over_algorithmic"] = load_pmc(f"osr{osr}_sf7", "step_traffic_over_algorithmic")
            if rt is not None:
                line["three_launch"] = {"ms_per_step": rt["ms_per_step"], "stage_ms": rt["stage_ms"],
                                        "pipeline_frac": rt["pipeline_gbs"] / HBM_PEAK_GBS,
                                        "symbols_ok": rt["symbols_ok"], "kernels": rt["kernels"]}
                del rt
            extra[f"osr{osr}_sf7"] = line
            del ro
            torch.cuda.empty_cache()
        # the reference's two other receivers on the headline's shape: the workspace API's
        # demodulate (phy.cpp:178-239, rx_runner's path: estimate on raw samples, fused
        # per-symbol down-chirp) and the detector alone (tests/awgn_sweep.py:262-273); each
        # with its own roofline and a reference leg (rate + parity on a 32-frame sample)
        for mode, note in (("api", "workspace API demodulate (phy.cpp:178-239) on raw modulated frames; "
                                   "ser_vs_tx is the reference's own estimate-on-raw-samples behaviour"),
                           ("raw", "detector only per symbol (awgn_sweep.py:262-273), all 66 symbols an output")):
            rm = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, dist, device, rank=rank,
                            mode=mode, inputs=(r7["syms"], r7["iq"]))
            leg = None
            if rank == 0 and world == 1 and not args.no_cpu:
                try:
                    leg = reference_leg(rm)
                except Exception as e:  # the CPU leg must not kill the GPU measurement
                    log(f"{mode} reference leg failed:", e)
            line = variant_summary(rm, r7, note, {"parity_ok": leg["parity_ok"] if leg else None,
                                                  "vs": "cpu_baseline leg (reference outputs on its sample)"})
            line["roofline"] = roofline(rm, probe)
            line["cpu_baseline"] = leg
            extra[f"{mode}_sf7"] = line
            del rm
        extra["mod_sf7"] = run_modulator(7, args.frames, args.data_symbols, device,
                                         with_cpu=rank == 0 and not args.no_cpu)
    r12 = None
    if not args.no_sf12:
        r12 = run_config(12, args.sf12_frames, args.data_symbols, max(args.steps // 2, 2),
                         args.warmup, dist, device, rank=rank)
        extra["sf12"] = public(r12)
        extra["sf12"]["value_all_ranks_msym_s"] = r12["msym_s_all_ranks"]
        extra["sf12"]["roofline"] = roofline(r12, probe)
        extra["sf12"]["parity"] = exact_parity(r12, device)
        if not args.no_fast:
            r12f = run_config(12, args.sf12_frames, args.data_symbols, max(args.steps // 2, 2), args.warmup,
                              dist, device, precision="fast", inputs=(r12["syms"], r12["iq"]), rank=rank)
            extra["fast_rotation_sf12"] = fast_summary(r12f, r12)
            del r12f
        if rank == 0 and not args.no_cpu and world == 1:
            try:
                extra["sf12"]["cpu_baseline"] = cpu_baseline(12, r12["iq"], args.data_symbols, 64,
                                                             gpu_out=r12["out"])
            except Exception as e:  # the CPU leg must not kill the GPU measurement
                log("sf12 cpu baseline failed:", e)
        if not args.no_variants:
            # noisy copy of the same batch, generated in place (no second 33.8 GB buffer)
            sigma = 10.0 ** (10.0 / 20.0) / math.sqrt(2.0)
            gn = torch.Generator(device=device).manual_seed(77)
            iqn = r12["iq"]
            for r0 in range(0, iqn.shape[0], 512):
                blk = iqn[r0:r0 + 512]
                blk += torch.view_as_complex(torch.randn(blk.shape + (2,), generator=gn, device=device)) * sigma
            r12n = run_config(12, args.sf12_frames, args.data_symbols, max(args.steps // 4, 2), args.warmup,
                              dist, device, inputs=(r12["syms"], iqn), rank=rank)
            extra["awgn_m10db_sf12"] = variant_summary(r12n, r12, "AWGN -10 dB on the SF12 batch: symbol errors "
                                                                  "and near-ties, recomputed exactly",
                                                       exact_parity(r12n, device))
            del r12n
        del r12
        torch.cuda.empty_cache()
        if not args.no_variants:
            # the SF12 batch's shape (15,625 frames): the modulator's time is set by each
            # frame's sequential phase chain (k_mod_phase), so a smaller batch only measures
            # that chain's length
            extra["mod_sf12"] = run_modulator(12, args.sf12_frames, args.data_symbols, device,
                                              with_cpu=rank == 0 and not args.no_cpu)
    if not args.no_channels:
        extra["channels"] = run_channels(args.channel_frames, 16, max(args.steps // 4, 2), 1, dist, device, rank)
        torch.cuda.empty_cache()
    cpu = None
    if rank == 0 and not args.no_cpu and world == 1:
        try:
            cpu = cpu_baseline(7, r7["iq"], args.data_symbols, 4000, gpu_out=r7["out"])
        except Exception as e:  # the CPU leg must not kill the GPU measurement
            log("cpu baseline failed:", e)
    if rank == 0:
        workload = (f"SF7 BW125 osr1 LEGACY lora_demodulate + fused dechirp, {args.frames} frames x "
                    f"(2 sync + {args.data_symbols} data) symbols per GPU, noiseless")
        line = {
            "metric": METRIC,
            "value": r7["msym_s_all_ranks"],
            "unit": "Msymbols/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": r7["ms_per_step_max_rank"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (GPU lora_modulate of seeded random symbols, amplitude 1, no noise)",
            "config": {"workload": workload, "launch": LAUNCH, "prewarm_ms": PREWARM_MS,
                       "streams": r7["streams"], "one_stream": one, "sf": 7, "bw_hz": 125000,
                       "osr": 1,
                       "frames_per_gpu": args.frames, "data_symbols_per_frame": args.data_symbols,
                       "parallelism": f"frames sharded x{world}, no collective (gloo timing only)",
                       "ranks": ranks, "symbols_ok": r7["symbols_ok"], "parity": r7["parity"],
                       "stage_ms": r7["stage_ms"], "stage_ms_streams": r7["stage_ms_streams"],
                       "kernels": r7["kernels"], "spec_recomputed_per_step": r7["spec_recomputed_per_step"],
                       "msym_s_all_symbols": r7["msym_s_all"] * world,
                       "pipeline_gbs_per_gpu": r7["pipeline_gbs"]},
            "roofline": roofline(r7, probe),
            "cpu_baseline": cpu,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
