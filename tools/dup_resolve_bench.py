"""Time of distributed.resolve_cross_shard_duplicates, the step every
read-sharded job (config 3 / config 5 shards) runs before its totals
(ADVICE r4), over gloo on the CPU:

    python tools/dup_resolve_bench.py --world 2 --reads 12500000 [--dup-frac 0.01]

Each rank holds a shard of `--reads` ids ("read_<global index>", as a FASTQ
of config 3 names them) with a D-column uint8 hit matrix; `--dup-frac` of
them repeat an id of the next rank's shard.  Prints one JSON line per rank 0
with every rank's time and the rows dropped.  (The collectives here are
gloo's; under RCCL the all-to-alls run on device tensors.)
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]


def _ids(lo: int, hi: int):
    sys.path.insert(0, str(ROOT))
    from xspect2_amd.packing import PackedIds
    # "read_<i>" for i in [lo, hi), packed without a Python string per id
    nums = np.arange(lo, hi, dtype=np.int64)
    digits = np.floor(np.log10(np.maximum(nums, 1))).astype(np.int64) + 1
    lens = 5 + digits
    offs = np.zeros(nums.size + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    buf = np.empty(int(offs[-1]), dtype=np.uint8)
    starts = offs[:-1].astype(np.int64)
    for j, c in enumerate(b"read_"):
        buf[starts + j] = c
    for d in range(int(digits.max()) if nums.size else 0):  # digit d from the right
        has = digits > d
        pos = starts[has] + 5 + digits[has] - 1 - d
        buf[pos] = ord("0") + (nums[has] // 10 ** d) % 10
    return PackedIds(buf.tobytes(), offs)


def _rank(rank: int, world: int, port: int, n: int, dup: float, D: int, out: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    from xspect2_amd import distributed
    from xspect2_amd.result import MatrixResult

    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo = rank * n
    ids = _ids(lo, lo + n)
    m = int(dup * n)
    if m and world > 1:  # this shard's first m ids repeat ids m..2m-1 of the next rank's shard
        nb = ((rank + 1) % world) * n
        nxt = _ids(nb + m, nb + 2 * m)
        ids = type(ids).concat([nxt, ids.take(np.arange(m, n))])
    hits = np.random.default_rng(rank).integers(0, 131, (n, D), dtype=np.uint8)
    res = MatrixResult("bench", ids, [f"d{i}" for i in range(D)], hits, np.full(n, 130, np.uint64))
    dist.barrier()
    t = time.perf_counter()
    dropped = distributed.resolve_cross_shard_duplicates(res)
    dt = time.perf_counter() - t
    allr: list = [None] * world
    dist.all_gather_object(allr, {"rank": rank, "s": dt, "dropped": dropped, "rows_after": len(res.ids)})
    if rank == 0:
        Path(out).write_text(json.dumps({"world": world, "reads_per_rank": n, "dup_frac": dup, "docs": D,
                                         "max_s": max(r["s"] for r in allr), "per_rank": allr}))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--reads", type=int, default=1_000_000, help="ids per rank")
    ap.add_argument("--dup-frac", type=float, default=0.0)
    ap.add_argument("--docs", type=int, default=8)
    a = ap.parse_args()
    import tempfile

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tempfile.mktemp(suffix=".json")
    mp.spawn(_rank, args=(a.world, port, a.reads, a.dup_frac, a.docs, out), nprocs=a.world, join=True)
    print(Path(out).read_text())


if __name__ == "__main__":
    main()
