"""Per-call time of all_gather_into_tensor of one band (one rank here: the
collective's launch + completion latency on the communication stream)."""
import os, sys, time
import torch
import torch.distributed as dist
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
for nb in (800_000, 1_600_000, 6_400_000):
    x = torch.empty(nb, dtype=torch.uint8, device="cuda")
    y = torch.empty(nb * dist.get_world_size(), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    for _ in range(20):
        with torch.cuda.stream(s):
            dist.all_gather_into_tensor(y, x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    K = 200
    with torch.cuda.stream(s):
        for _ in range(K):
            dist.all_gather_into_tensor(y, x)
    torch.cuda.synchronize()
    print(f"bytes {nb}: {1e6 * (time.perf_counter() - t0) / K:.1f} us per all_gather", flush=True)
dist.destroy_process_group()
