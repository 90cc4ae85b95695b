"""Can two RCCL ranks share one GPU on this pool?  (one-GPU box rehearsal aid)

Started by tools/gpu/gpu_r04_launch.sh under bench-style env (RANK, WORLD_SIZE,
MASTER_*): init_process_group("nccl") on cuda:0 in both ranks, one all-reduce
and one uint8 all-gather, then report.  A refusal (RCCL's duplicate-device
check) or any error is printed and the rank exits 1."""
import os
import sys

import torch
import torch.distributed as dist

r = int(os.environ["RANK"])
w = int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
try:
    dist.init_process_group("nccl", device_id=dev)
    t = torch.ones(4, device=dev) * (r + 1)
    dist.all_reduce(t)
    g = [torch.empty(8, dtype=torch.uint8, device=dev) for _ in range(w)]
    dist.all_gather(g, torch.full((8,), r, dtype=torch.uint8, device=dev))
    torch.cuda.synchronize()
    ok = t[0].item() == w * (w + 1) / 2 and all(int(x[0].item()) == i for i, x in enumerate(g))
    print(f"rank {r}: RCCL world {dist.get_world_size()} on one GPU: all_reduce {t[0].item()} gather ok={ok}",
          file=sys.stderr, flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 2)
except Exception as e:  # noqa: BLE001
    print(f"rank {r}: RCCL on a shared GPU refused: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
    sys.exit(1)
