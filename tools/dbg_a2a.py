"""all_to_all_single on a one-rank RCCL group: is a large buffer copied intact?"""
import os
import sys
import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29556")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for lg in (26, 27, 28, 29):
    for dt in (torch.int64, torch.int32):
        n = (1 << lg) + 12345
        a = torch.arange(n, device="cuda").to(dt)
        b = torch.zeros_like(a)
        dist.all_to_all_single(b, a)
        torch.cuda.synchronize()
        bad = (a != b).nonzero()
        print(lg, dt, n * a.element_size() / 2**30, "GiB", "bad", bad.numel(),
              int(bad[0].item()) if bad.numel() else -1, flush=True)
        del a, b
dist.destroy_process_group()
