"""Probe: can several RCCL ranks share ONE GPU (to rehearse multi-rank RCCL paths
on a 1-GPU box)? Each rank uses cuda:0; runs all_gather / all_to_all / send-recv."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    x = torch.full((world, 1024), float(rank), device=dev)
    dist.all_gather_into_tensor(x.view(-1), x[rank])
    a = torch.arange(world * 4, device=dev, dtype=torch.float32) + 100 * rank
    b = torch.empty_like(a)
    dist.all_to_all_single(b, a)
    ops = []
    peer = (rank + 1) % world
    src = (rank - 1) % world
    s = torch.full((8,), float(rank), device=dev)
    r = torch.empty(8, device=dev)
    ops.append(dist.P2POp(dist.isend, s, peer))
    ops.append(dist.P2POp(dist.irecv, r, src))
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    torch.cuda.synchronize()
    ok = bool((x[:, 0].cpu() == torch.arange(world).float()).all()) and float(r[0]) == src
    print(f"rank {rank}: allgather+a2a+p2p ok={ok} a2a={b.cpu().tolist()[:8]}", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
