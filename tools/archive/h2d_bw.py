"""H2D bandwidth from pinned host memory on 1, 2 and 4 streams (diagnostics,
GPU): the device reader's text load is one H2D stream of 4 MiB pieces."""
import json
import time

import torch


def run(nbytes, streams, piece=4 << 20, reps=5):
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ss = [torch.cuda.Stream() for _ in range(streams)]
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i, o in enumerate(range(0, nbytes, piece)):
            with torch.cuda.stream(ss[i % streams]):
                dst[o:o + piece].copy_(src[o:o + piece], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return nbytes / best / 1e9


out = {}
for mb in (64, 256):
    for s in (1, 2, 4):
        out[f"{mb}MiB_{s}streams_GBps"] = round(run(mb << 20, s), 2)
print(json.dumps(out))
