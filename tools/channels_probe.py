"""configs[4] chunking probe: bench.run_channels (1e6 SF7 frames of 2 + 16 symbols, resident)
at several chunk sizes, alternated, one process.  usage: python tools/channels_probe.py [GB ...]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402

sizes = [float(x) for x in sys.argv[1:]] or [8.0, 4.0, 2.0]
dev = torch.device("cuda", 0)
for rep in range(2):
    for gb in sizes:
        r = bench.run_channels(1_000_000, 16, 20, 2, None, dev, 0, chunk_bytes=gb * 1e9)
        print(json.dumps({"rep": rep, "chunk_gb": gb, "chunks": r["chunks"], "ms_per_step": round(r["ms_per_step"], 4),
                          "msym_s": round(r["value_all_ranks_msym_s"], 1), "ok": r["symbols_ok_all_frames"]}), flush=True)
        torch.cuda.empty_cache()
