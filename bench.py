"""Benchmark: LoRa demod hot path (dechirp -> 2^SF FFT -> argmax) on MI355X.

One step = one lora_demod_batch over this rank's batch of frames already resident in
HBM: LEGACY lora_demodulate semantics with the fused caller-side dechirp
(e2e_chain_test.cpp:85-101): normalisation, 2-symbol CFO/timing estimate, per-symbol
CFO rotation, FFT, argmax, sync word.  Inputs are generated on the device by the
bit-exact GPU modulator (lora_mod_batch), random symbols from a fixed seed.

Headline workload (BASELINE.json configs[1]): SF7 BW125 osr 1, 1,000,000 data symbols
= 15,625 frames x (2 sync + 64 data) per GPU.  The SF12 configuration (configs[2]) is
measured in the same run and reported under "extra".  Multi-GPU: one process per GPU,
frames sharded (no collective on the data path), weak scaling; value = data symbols of
all ranks / max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lora-sdr-lightweight-standalone-library-_amd"))
sys.path.insert(0, REPO)

import lora_phy_amd as amd  # noqa: E402
from lora_phy_amd import _capi  # noqa: E402
from lora_phy_amd.shard import aggregate_throughput  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
METRIC = "Msymbols/s dechirp+FFT+argmax @ SF7 & SF12, 1/2/4/8 GPU; % HBM roofline"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup(n_gpus):
    """One process per GPU (torchrun).  The collectives are only the timing barrier and
    the max/sum all-reduces (lora_phy_amd.shard); frames never cross GPUs.  Backend
    "nccl" (RCCL) by default; LORA_BENCH_BACKEND=gloo rehearses the multi-rank path with
    several ranks on fewer GPUs (ranks share devices round-robin)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist

        local = int(os.environ.get("LOCAL_RANK", "0"))
        backend = os.environ.get("LORA_BENCH_BACKEND", "nccl")
        dev = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        return dist, dist.get_rank(), world
    torch.cuda.set_device(0)
    return None, 0, 1


SYNC = 0x12


def make_input(sf, frames, data_syms, seed, device, snr_db=None):
    g = torch.Generator(device="cpu").manual_seed(seed)
    syms = torch.randint(0, 1 << sf, (frames, data_syms), generator=g, dtype=torch.int32)
    iq = amd.modulate(syms.to(device), sf, 1, 125000, 1.0, SYNC)
    if snr_db is not None:
        sigma = 10.0 ** (-snr_db / 20.0) / np.sqrt(2.0)
        gn = torch.Generator(device=device).manual_seed(seed + 1)
        noise = torch.randn(iq.shape + (2,), generator=gn, device=device) * sigma
        iq = iq + torch.view_as_complex(noise)
    return syms, iq


def run_config(sf, frames, data_syms, steps, warmup, rank, dist, device, snr_db=None, precision="exact",
               inputs=None):
    N = 1 << sf
    syms, iq = inputs if inputs is not None else make_input(sf, frames, data_syms, 20251015 + rank, device,
                                                            snr_db)
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, mode="legacy", device=device,
                         precision=precision)
    out = None
    for _ in range(warmup):
        out = plan.run(iq, out)
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        out = plan.run(iq, out)
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    # Per-kernel durations: a second pass of the same steps with HIP events around every
    # launch, recorded on the stream each kernel runs on (not inside the timed region).
    import ctypes as C

    lib = _capi.lib()
    _capi.check(lib.lora_demod_profile_enable(plan._h, steps))
    for _ in range(steps):
        out = plan.run(iq, out)
    torch.cuda.synchronize(device)
    stage = (C.c_float * 3)()
    calls = C.c_int()
    _capi.check(lib.lora_demod_profile_read(plan._h, stage, C.byref(calls)))
    lib.lora_demod_profile_enable(plan._h, 0)
    stage_ms = [stage[k] / max(calls.value, 1) for k in range(3)]
    # weak scaling: every rank owns its frames; units summed, time = max over ranks
    units, wall, _ = aggregate_throughput(frames * data_syms * steps, wall)
    ok = bool(torch.equal(out.symbols.to(torch.int32).cpu(), syms)) if snr_db is None else None
    total_syms = data_syms + 2
    ms_step = wall * 1e3 / steps
    B_sym = 8 * N + 2
    # Dominant kernel = stage 2 (k_demod: every non-sync symbol).  Algorithmic bytes
    # per launch = its symbols x (8*N*osr IQ read + 2 B index write).
    demod_bytes = frames * data_syms * B_sym
    dom_gbs = demod_bytes / (stage_ms[2] * 1e-3) / 1e9
    pipe_bytes = frames * (total_syms * B_sym + 9)
    return {
        "sf": sf, "frames": frames, "data_symbols": frames * data_syms, "iq_bytes": iq.numel() * 8,
        "ms_per_step": ms_step, "stage_ms": stage_ms, "symbols_ok": ok,
        "msym_s_data": frames * data_syms / (ms_step * 1e-3) / 1e6,
        "msym_s_all_ranks": units / wall / 1e6,
        "msym_s_all": frames * total_syms / (ms_step * 1e-3) / 1e6,
        "dominant_kernel": "k_demod", "dominant_gbs": dom_gbs,
        "dominant_bytes_per_launch": demod_bytes,
        "pipeline_gbs": pipe_bytes / (ms_step * 1e-3) / 1e9,
        "iq_host": None, "plan": plan, "iq": iq, "syms": syms,
    }


def run_channels(frames, data_syms, steps, warmup, rank, dist, device, chunk_bytes=8e9):
    """BASELINE.json configs[4]: one channel per GPU, `frames` SF7 frames of 2 + `data_syms`
    symbols resident in HBM (18.4 GB at 1e6 x 16), demodulated in <= 8 GB chunks per step
    (SURVEY.md 8d item 5).  Inputs generated on the device (GPU modulator) in slices."""
    sf, N = 7, 128
    L = (data_syms + 2) * N
    iq = torch.empty((frames, L), dtype=torch.complex64, device=device)
    g = torch.Generator(device="cpu").manual_seed(4242 + rank)
    gen_rows = 1 << 17
    first_syms = None
    for r0 in range(0, frames, gen_rows):
        n = min(gen_rows, frames - r0)
        syms = torch.randint(0, N, (n, data_syms), generator=g, dtype=torch.int32)
        if first_syms is None:
            first_syms = syms[:64].clone()
        iq[r0:r0 + n] = amd.modulate(syms.to(device), sf, 1, 125000, 1.0, SYNC)
    plan = amd.DemodPlan(sf, 1, 125000, "none", dechirp=True, mode="legacy", device=device)
    per_chunk = max(1, int(chunk_bytes // (L * 8)))
    chunks = [(c0, min(per_chunk, frames - c0)) for c0 in range(0, frames, per_chunk)]
    outs = [None] * len(chunks)

    def step():
        for i, (c0, n) in enumerate(chunks):
            outs[i] = plan.run(iq[c0:c0 + n], outs[i])

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    units, wall_max, _ = aggregate_throughput(frames * data_syms * steps, wall)
    ok = bool(torch.equal(outs[0].symbols[:64].to(torch.int32).cpu(), first_syms))
    del iq
    return {"frames_per_gpu": frames, "data_symbols_per_frame": data_syms, "iq_gb_per_gpu": frames * L * 8 / 1e9,
            "chunks": len(chunks), "ms_per_step": wall_max * 1e3 / steps,
            "value_all_ranks_msym_s": units / wall_max / 1e6, "symbols_ok_first64": ok}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sf, iq_dev, data_syms, max_frames, threads, time_budget_s=10.0):
    """The reference's own lora_demodulate (oracle/_ref, compiled from the reference's
    sources, travels with the snapshot) on `threads` host cores over a bounded sample of
    the same frames; falls back to the restatement (oracle/lora_oracle.cpp) if absent.
    Reported `value`: all threads, caller-side dechirp + lora_demodulate (the GPU
    workload).  Also: one core, and demod only (input dechirped beforehand), per
    SURVEY.md 8d.  The reported leg: whole passes over the sample until `time_budget_s`
    (about 10 s of CPU work); the single-core and demod-only legs: half that."""
    from oracle.pyoracle import Oracle, Reference

    if Reference.available():
        impl, kind, what = Reference(), "reference", "reference src/phy lora_demodulate (oracle/_ref)"
    else:
        impl, kind, what = Oracle(), "port", "restatement oracle/lora_oracle.cpp"
    F = min(iq_dev.shape[0], max_frames)
    x = iq_dev[:F].cpu().numpy()

    def rate(xs, nthreads, dechirp, budget):
        impl.demod_frames(xs[: min(len(xs), 4 * nthreads)], sf, 1, False, dechirp=dechirp, threads=nthreads)
        t0 = time.perf_counter()
        done = 0
        while True:
            impl.demod_frames(xs, sf, 1, False, dechirp=dechirp, threads=nthreads)
            done += len(xs)
            if time.perf_counter() - t0 > budget:
                break
        dt = time.perf_counter() - t0
        return done * data_syms / dt / 1e6, done, dt

    all_rate, done, dt = rate(x, threads, True, time_budget_s)
    one_rate, _, _ = rate(x[: max(1, F // max(threads, 1))], 1, True, time_budget_s / 2)
    xd = Oracle().dechirp(x.reshape(-1), sf).reshape(x.shape)  # same fp32 products as the caller loop
    demod_only, _, _ = rate(xd, threads, False, time_budget_s / 2)
    return {"value": all_rate, "unit": "Msymbols/s", "cores": threads, "kind": kind,
            "single_core": one_rate, "demod_only_all_cores": demod_only, "cpu_model": _cpu_model(),
            "sample": f"{done} frames of the SF{sf} bench batch ({data_syms}+2 symbols each), "
                      f"caller-side dechirp + {what}, {threads} threads, {dt:.2f} s; single_core: same "
                      f"on 1 thread; demod_only: input dechirped beforehand"}


def fast_summary(r):
    """LORA_PRECISION_FAST line (hardware sin/cos rotation; stated tolerance in
    include/lora_mi355x.h): same workload and inputs as the exact run."""
    return {"precision": "fast", "ms_per_step": r["ms_per_step"], "stage_ms": r["stage_ms"],
            "symbols_ok": r["symbols_ok"], "value_all_ranks_msym_s": r["msym_s_all_ranks"],
            "demod_gbs": r["dominant_gbs"], "demod_roofline_frac": r["dominant_gbs"] / HBM_PEAK_GBS}


def hbm_probe(device, nbytes=2 << 30, reps=5):
    """SURVEY.md 8d cross-check: device-to-device copy bandwidth on the same GPU
    (bytes read + bytes written per second), the chip's achievable HBM rate next to the
    8 TB/s spec."""
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


def valu_roofline(workload, kernel_ms):
    """The demod kernel's real limit: VALU issue.  Counts from the committed PMC profile
    (profiles/pmc_summary.json, same kernel and workload) against the live kernel time;
    peak = the time the profiled fp32/fp64 instruction mix needs at the chip's measured
    issue rates (tools/micro/pk_rate)."""
    v = load_pmc(workload, "valu_winstr_per_launch")
    need = load_pmc(workload, "valu_mix_ns_cu")
    if not v or not need or not kernel_ms:
        return None
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    achieved = v / (kernel_ms * 1e6) / ncu  # wave-instructions per ns per CU
    return {"bound": "valu-issue", "winstr_per_launch": v,
            "fp64_class_per_launch": load_pmc(workload, "valu_fp64_class_per_launch"),
            "achieved_winstr_per_ns_per_cu": achieved,
            "frac": need / ncu / (kernel_ms * 1e6),
            "note": "frac = (profiled instruction mix at measured peak issue rates) / live kernel time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=15625)
    ap.add_argument("--data-symbols", type=int, default=64)
    ap.add_argument("--sf12-frames", type=int, default=15625)
    ap.add_argument("--no-sf12", action="store_true")
    ap.add_argument("--sf12-only", action="store_true", help="profiling: SF12 workload only")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-channels", action="store_true", help="skip the configs[4] measurement")
    ap.add_argument("--no-fast", action="store_true", help="skip the LORA_PRECISION_FAST lines")
    ap.add_argument("--channel-frames", type=int, default=1_000_000)
    ap.add_argument("--cpu-threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--sync", type=lambda v: int(v, 0), default=0x12,
                    help="sync word of the synthetic frames (0x12 = the reference default; "
                         "large nibbles -> large estimated CFO -> phases past the fast sincos range)")
    args = ap.parse_args()
    global SYNC
    SYNC = args.sync

    dist, rank, world = dist_setup(args.gpus)
    device = torch.device("cuda", torch.cuda.current_device())
    if args.sf12_only:
        r12 = run_config(12, args.sf12_frames, args.data_symbols, args.steps, args.warmup, rank, dist,
                         device)
        if rank == 0:
            print(json.dumps({k: v for k, v in r12.items() if k not in ("plan", "iq", "iq_host", "syms")}))
        return
    r7 = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, rank, dist, device)
    extra = {}
    if not args.no_fast:
        r7f = run_config(7, args.frames, args.data_symbols, args.steps, args.warmup, rank, dist, device,
                         precision="fast", inputs=(r7["syms"], r7["iq"]))
        extra["fast_rotation_sf7"] = fast_summary(r7f)
        del r7f
    if not args.no_sf12:
        r12 = run_config(12, args.sf12_frames, args.data_symbols, max(args.steps // 2, 2),
                         args.warmup, rank, dist, device)
        extra["sf12"] = {k: v for k, v in r12.items() if k not in ("plan", "iq", "iq_host", "syms")}
        extra["sf12"]["value_all_ranks_msym_s"] = r12["msym_s_all_ranks"]
        extra["sf12"]["roofline_frac"] = r12["dominant_gbs"] / HBM_PEAK_GBS
        extra["sf12"]["traffic"] = load_pmc("sf12")
        extra["sf12"]["valu"] = valu_roofline("sf12", r12["stage_ms"][2])
        extra["sf12"]["frame_max_read_gbs"] = r12["iq_bytes"] / (r12["stage_ms"][0] * 1e-3) / 1e9
        if not args.no_fast:
            r12f = run_config(12, args.sf12_frames, args.data_symbols, max(args.steps // 2, 2), args.warmup, rank,
                              dist, device, precision="fast", inputs=(r12["syms"], r12["iq"]))
            extra["fast_rotation_sf12"] = fast_summary(r12f)
            del r12f
        del r12
        torch.cuda.empty_cache()
    if not args.no_channels and not args.sf12_only:
        extra["channels"] = run_channels(args.channel_frames, 16, max(args.steps // 4, 2), 1, rank, dist,
                                         device)
        torch.cuda.empty_cache()
    probe = None
    try:
        probe = hbm_probe(device)
    except Exception as e:  # a probe must not kill the measurement
        log("hbm probe failed:", e)
    cpu = None
    if rank == 0 and not args.no_cpu and world == 1:
        try:
            cpu = cpu_baseline(7, r7["iq"], args.data_symbols, 4000, args.cpu_threads)
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
            "ms_per_step": r7["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (GPU lora_modulate of seeded random symbols, amplitude 1, no noise)",
            "config": {"workload": workload, "sf": 7, "bw_hz": 125000, "osr": 1,
                       "frames_per_gpu": args.frames, "data_symbols_per_frame": args.data_symbols,
                       "parallelism": f"frames sharded x{world}, no collective",
                       "symbols_ok": r7["symbols_ok"], "stage_ms": r7["stage_ms"],
                       "msym_s_all_symbols": r7["msym_s_all"] * world,
                       "pipeline_gbs_per_gpu": r7["pipeline_gbs"]},
            "roofline": {"bound": "hbm", "kernel": r7["dominant_kernel"],
                         "achieved": r7["dominant_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": r7["dominant_gbs"] / HBM_PEAK_GBS,
                         "bytes_per_launch": r7["dominant_bytes_per_launch"],
                         "traffic": load_pmc("sf7"),
                         "valu": valu_roofline("sf7", r7["stage_ms"][2]),
                         "hbm_probe": {"d2d_copy_gbs": probe,
                                       "frame_max_read_gbs": r7["iq_bytes"] / (r7["stage_ms"][0] * 1e-3) / 1e9,
                                       "note": "achievable rates on this GPU: torch D2D copy (read+write) and "
                                               "the k_frame_max streaming read of the same IQ"}},
            "cpu_baseline": cpu,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
