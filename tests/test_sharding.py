"""CPU, world_size 2 over gloo: the frame-sharded multi-GPU path (lora_phy_amd.shard).

Each rank takes its shard_range block of a seeded global batch, demodulates it (here
with the CPU oracle standing in for the GPU kernel, which needs a device), and the
results are gathered and compared with the whole batch demodulated in one process.
aggregate_throughput must give sum(units) / max(seconds) - the bench.py contract.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lora_phy_amd.shard import aggregate_throughput, gather_frames, shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 15625):
        for world in (1, 2, 3, 8):
            blocks = [shard_range(n, r, world) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            for (a, b), (c, d) in zip(blocks, blocks[1:]):
                assert b == c
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def global_batch(O, sf, F, S):
    rng = np.random.default_rng(404)
    syms = rng.integers(0, 1 << sf, (F, S)).astype(np.uint16)
    rows = []
    for f in range(F):
        x = O.lora_modulate(syms[f], sf)
        x = (x + 0.4 * (rng.standard_normal(len(x)) + 1j * rng.standard_normal(len(x)))).astype(np.complex64)
        rows.append(x)
    return syms, np.stack(rows)


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.pyoracle import Oracle

        O = Oracle()
        sf, F, S = 7, 13, 6
        _, iq = global_batch(O, sf, F, S)
        a, b = shard_range(F, rank, world)
        syms, sync, cfo, toff, _ = O.demod_frames(iq[a:b], sf, dechirp=True)
        local = torch.from_numpy(syms[:, :S].astype(np.int32))
        full = gather_frames(local, F)
        full_sync = gather_frames(torch.from_numpy(sync), F)
        full_cfo = gather_frames(torch.from_numpy(cfo), F)
        units, secs, value = aggregate_throughput(local.numel(), 0.5 + rank)
        if rank == 0:
            json.dump({"syms": full.tolist(), "sync": full_sync.tolist(),
                       "cfo": full_cfo.numpy().view(np.uint32).tolist(),
                       "units": units, "secs": secs, "value": value}, open(out_path, "w"))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharded_demod(tmp_path):
    from oracle.pyoracle import Oracle

    out = str(tmp_path / "r0.json")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = json.load(open(out))
    O = Oracle()
    sf, F, S = 7, 13, 6
    tx, iq = global_batch(O, sf, F, S)
    syms, sync, cfo, _, _ = O.demod_frames(iq, sf, dechirp=True)
    np.testing.assert_array_equal(np.array(got["syms"]), syms[:, :S])
    np.testing.assert_array_equal(np.array(got["syms"]), tx)  # 0.4 noise: loopback exact
    np.testing.assert_array_equal(np.array(got["sync"]), sync)
    np.testing.assert_array_equal(np.array(got["cfo"], np.uint32), cfo.view(np.uint32))
    assert got["units"] == F * S
    assert got["secs"] == 1.5  # max over ranks, not the sum or mean
    assert got["value"] == F * S / 1.5


def test_single_process_aggregate_is_local():
    assert not dist.is_initialized()
    assert aggregate_throughput(100, 2.0) == (100.0, 2.0, 50.0)
    t = torch.arange(6).reshape(3, 2)
    assert gather_frames(t, 3) is t
