"""Probe: can two RCCL ranks share one GPU (for rehearsing bench.py's RCCL gather on a
one-GPU box)?  Prints the outcome of one dist.gather; diagnostic only."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((4,), float(rank), device="cuda")
    out = [torch.empty(4, device="cuda") for _ in range(2)] if rank == 0 else None
    dist.gather(x, gather_list=out, dst=0)
    torch.cuda.synchronize()
    print(f"rank {rank}: gather ok", [t.tolist() for t in out] if out else "", flush=True)
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001
    print(f"rank {rank}: {type(e).__name__}: {str(e)[:300]}", flush=True)
