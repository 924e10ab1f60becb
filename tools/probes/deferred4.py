"""Probe: the 4-rank deferred-union-check step on one card (gloo, CUDA tensors), with a CPU all_gather
reference of the dense SUM on every rank (round 5: ranks disagreed on the dense all-reduce)."""
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def worker(rank, world, port, P, V, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams
    from dge_amd.multiview import GradBucket, render_views, shard_views
    from dge_amd.scene import synthetic_scene

    sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
    cams = [orbit_camera(k, 24, W, H, device=dev) for k in range(V)]
    g = torch.Generator().manual_seed(7)
    seeds = [(torch.randn(3, H, W, generator=g) * 1e-3).to(dev) for _ in range(V)]
    mine = list(shard_views(V, world, rank))
    bucket = GradBucket(sc.parameters())
    bg = torch.zeros(3, device=dev)
    lines = []
    for step in range(2):
        bucket.zero()
        outs = render_views([cams[i] for i in mine], sc, PipelineParams(), bg, streams=3, speculate=True)
        bucket.allreduce_begin([o["_live_rows"] for o in outs], min_world=2)
        torch.autograd.backward([o["render"] for o in outs], [seeds[i] for i in mine])
        ok = outs.check()
        torch.cuda.synchronize()
        local = bucket.flat.cpu()
        dense = bucket.flat.clone()
        dist.all_reduce(dense, op=dist.ReduceOp.SUM)
        torch.cuda.synchronize()
        gathered = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(gathered, local)
        ref = gathered[0].clone()
        for t in gathered[1:]:
            ref += t
        d = dense.cpu()
        lines.append(dict(step=step, mine=mine, ok=ok, local_nz=int((local != 0).sum()), dense_nz=int((d != 0).sum()),
                          ref_nz=int((ref != 0).sum()), dense_vs_ref=float((d - ref).abs().max()),
                          pending=str(bucket._pending[0]) if getattr(bucket, "_pending", None) else None))
        bucket.allreduce_end(defer_check=True)
        bucket.allreduce_finalize()
        torch.cuda.synchronize()
        f = bucket.flat.cpu()
        lines[-1].update(packed_vs_ref=float((f - ref).abs().max()), packed_nz=int((f != 0).sum()))
    q.put((rank, lines))
    dist.destroy_process_group()


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    V = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, world, port, 300_000, V, 160, 128, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    for rank, lines in out:
        for ln in lines:
            print(rank, ln)
