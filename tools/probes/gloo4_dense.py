"""Probe: gloo all_reduce of CUDA tensors with 4 ranks on one card — is the SUM identical on every rank
and equal to the sum of the ranks' inputs gathered on the CPU?  (round 5: the 4-rank deferred-check test
saw ranks disagree on the dense all-reduce.)  Usage: python tools/probes/gloo4_dense.py [world]"""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    res = []
    for n, side in ((300_000 * 59, False), (300_000 * 59, True), (1_000_003, False)):
        g = torch.Generator().manual_seed(10 + rank)
        x = torch.zeros(n)
        idx = torch.randperm(n, generator=g)[: n // 5]
        x[idx] = torch.randn(idx.numel(), generator=g)
        xd = x.to(dev)
        if side:  # a MAX of a byte per row on a side stream first, as GradBucket.allreduce_begin does
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                live = (xd.reshape(-1, 59) != 0).any(1).to(torch.uint8)
                dist.all_reduce(live, op=dist.ReduceOp.MAX)
            torch.cuda.current_stream(dev).wait_stream(s)
        dense = xd.clone()
        dist.all_reduce(dense, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        gathered = [torch.zeros(n) for _ in range(world)]
        dist.all_gather(gathered, x)
        ref = sum(gathered[1:], gathered[0].clone()) if world > 1 else gathered[0]
        got = dense.cpu()
        res.append((n, side, float((got - ref).abs().max()), int((got != 0).sum()), int((ref != 0).sum()),
                    float(got.double().sum())))
    q.put((rank, res))
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for rank, res in out:
        print(rank, res)
