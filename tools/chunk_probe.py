#!/usr/bin/env python3
"""Probe (tool only): cost of cutting a rank's transform shard into chunks
(ShardedTable._overlapped on a one-rank RCCL group, so the all-gather is a
local copy and nothing overlaps): the price the N > 1 overlap must beat, at
the shard sizes of N = 2, 4, 8 (MIND-large dev, latent and final, bf16).

    python tools/chunk_probe.py > gpurun_out/chunks.jsonl
"""
import json
import os
import sys
import tempfile
from pathlib import Path

import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

from news_recommendation_project_v2_amd.distributed import ShardedTable  # noqa: E402
from news_recommendation_project_v2_amd.engine import PoolScoreEngine  # noqa: E402
from bench import make_model, news_table  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    store = os.path.join(tempfile.mkdtemp(), "store")
    dist.init_process_group("nccl", init_method=f"file://{store}", rank=0, world_size=1, device_id=dev)
    try:
        for pooler in ("latent", "final"):
            for world in (2, 4, 8):
                rows = (72023 + world - 1) // world
                eng = PoolScoreEngine(make_model(pooler, dev), dtype=torch.bfloat16, device=dev) \
                    .load_news(news_table(rows, dev))
                res = {"pooler": pooler, "world": world, "shard_rows": rows}
                for chunks in (1, 2, 3):
                    st = ShardedTable(eng, 0, 1, chunks=chunks)
                    for _ in range(3):
                        st._overlapped()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        st._overlapped()
                    e1.record()
                    torch.cuda.synchronize()
                    res[f"chunks{chunks}_ms"] = round(e0.elapsed_time(e1) / 10, 4)
                print(json.dumps(res), flush=True)
                del eng
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
