"""Multi-process (world_size 2, gloo, CPU) tests of the view-sharded step:
the sharded gradient bucket all-reduce and the densification statistics
reduce to exactly what the single-process loop over all views computes.

The per-view render here is the dense PyTorch formulation (tests/torch_ref.py)
so the data-parallel plumbing is checked end to end without a GPU; on the GPU
box the same code path runs with dge_amd's render() and the nccl (RCCL)
backend (bench.py --gpus N)."""
from __future__ import annotations

import datetime
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dge_amd.multiview import GradBucket, found_inf_allreduce, multiview_step, reduce_view_stats, shard_views


def test_shard_views_partition():
    for n in (1, 5, 24, 25):
        for w in (1, 2, 3, 8):
            shards = [list(shard_views(n, w, r)) for r in range(w)]
            flat = [i for s in shards for i in s]
            assert flat == list(range(n))
            assert max(map(len, shards)) - min(map(len, shards)) <= 1


class _Scene:
    """Minimal pc for the CPU render_fn: raw params + reference getters."""

    def __init__(self, P, seed):
        from dge_amd.scene import synthetic_scene

        sc = synthetic_scene(P, seed=seed, radius=1.0, scale=0.1, sh_degree=1)
        self.inner = sc.requires_grad_(True)

    def parameters(self):
        return self.inner.parameters()

    def num_points(self):
        return self.inner.num_points()


def _render_fn(cam, pc, pipe, bg):
    import torch_ref as TR
    from dge_amd.gaussian_renderer import _settings

    sc = pc.inner
    s = _settings(cam, bg, 1.0, sc.active_sh_degree)
    m2 = torch.zeros(sc.num_points(), 3, dtype=torch.float64, requires_grad=True)
    m2.retain_grad()
    c, _, radii, _ = TR.dense_render(sc.get_xyz, sc.get_opacity, s, shs=sc.get_features, scales=sc.get_scaling,
                                     rotations=sc.get_rotation, means2D=m2, dtype=torch.float64)
    return {"render": c.float(), "viewspace_points": _GradHolder(m2), "radii": torch.as_tensor(radii)}


class _GradHolder:
    def __init__(self, t):
        self.t = t

    @property
    def grad(self):
        return self.t.grad.float()


def _setup(P=60, V=4, W=32, H=32):
    from dge_amd.cameras import orbit_camera

    cams = [orbit_camera(k, V, W, H, device="cpu") for k in range(V)]
    g = torch.Generator().manual_seed(5)
    targets = [torch.randn(3, H, W, generator=g) for _ in range(V)]
    return cams, targets


def _step(pc, cams, targets, idx, V, mode):
    """multiview_step over views idx: gradient seeds (mode "seed") or DGE's masked l1 mean (mode "l1",
    targets = (gt images [3,H,W], masks [1,H,W]))."""
    bucket = GradBucket(pc.parameters())
    kw = dict(targets=[targets[i] for i in idx]) if mode == "seed" else dict(
        gt_images=[targets[0][i] for i in idx], masks=[targets[1][i] for i in idx], lambda_l1=10.0)
    out = multiview_step(pc, [cams[i] for i in idx], _render_fn, None, torch.zeros(3), bucket, V, **kw)
    return bucket, out


def _l1_targets(V, W=32, H=32):
    g = torch.Generator().manual_seed(9)
    gts = [torch.rand(3, H, W, generator=g) for _ in range(V)]
    masks = [(torch.rand(1, H, W, generator=g) > 0.3).float() for _ in range(V)]
    return gts, masks


def _worker(rank, world, port, P, V, mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["GLOO_SOCKET_IFNAME"] = "lo"  # (gloo on loopback: the host name need not resolve)
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    try:
        torch.set_num_threads(1)
        pc = _Scene(P, seed=4)
        cams, targets = _setup(P, V)
        if mode == "l1":
            targets = _l1_targets(V)
        bucket, out = _step(pc, cams, targets, list(shard_views(V, world, rank)), V, mode)
        # overflow on one rank only: every rank must see it (the GradScaler skip is collective)
        if rank == 1:
            bucket.flat[7] = float("nan")
        fi = found_inf_allreduce(bucket)
        q.put((rank, bucket.flat.clone().numpy() if rank == 0 else None, out["viewspace_grad_sum"].numpy(),
               out["radii_max"].numpy(), float(out["found_inf"].item()), float(fi.item())))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
@pytest.mark.parametrize("world,V", [(2, 4), (4, 10), (8, 24)], ids=["2ranks_4views", "4ranks_10views", "8ranks_24views"])
@pytest.mark.parametrize("mode", ["seed", "l1"])
def test_sharded_step_equals_single_process(mode, world, V):
    """world ranks x their shard_views shards == 1 process x V views (2 x 2 = 4; 4 ranks over 10 views: the
    uneven 3/3/2/2 shards; 8 ranks over c3's 24 views, 3 each: the driver's N = 8 shape): the summed parameter gradients (sparse-row bucket all-reduce), the view-space
    gradient sum and the radii max; for DGE's masked l1 (a mean over all views, DGE.py:672) through the
    B_local / B share of each rank.  found_inf is collective (a NaN on rank 1 only)."""
    P = 60
    pc = _Scene(P, seed=4)
    cams, targets = _setup(P, V)
    if mode == "l1":
        targets = _l1_targets(V)
    bucket, out = _step(pc, cams, targets, list(range(V)), V, mode)
    ref = bucket.flat.clone().numpy()
    vs1, r1 = out["viewspace_grad_sum"].numpy(), out["radii_max"].numpy()
    assert out["found_inf"].item() == 0.0 and np.abs(ref).max() > 0

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, P, V, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, flat, vs, rmax, fi_step, fi_nan in res:
        if flat is not None:
            np.testing.assert_allclose(flat, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
        np.testing.assert_allclose(vs, vs1, rtol=1e-5, atol=1e-6 * np.abs(vs1).max())
        np.testing.assert_array_equal(rmax, r1)
        assert fi_step == 0.0 and fi_nan == 1.0


def test_grad_bucket_views_and_zero():
    a = torch.zeros(3, 2, requires_grad=True)
    b = torch.zeros(5, requires_grad=True)
    bk = GradBucket([a, b])
    (a.sum() * 2 + (b * torch.arange(5.0)).sum()).backward()
    assert bk.check_attached()
    np.testing.assert_allclose(bk.flat.numpy(), [2] * 6 + [0, 1, 2, 3, 4])
    bk.zero()
    assert not bk.flat.any() and bk.check_attached()
    assert bk.allreduce() is None  # no process group: no-op
    vs, rm = reduce_view_stats(torch.ones(2, 3), torch.tensor([1, 2], dtype=torch.int32))
    assert vs.sum() == 6 and rm.tolist() == [1, 2]


def _sparse_worker(rank, world, port, q, row_major=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["GLOO_SOCKET_IFNAME"] = "lo"  # (gloo on loopback: the host name need not resolve)
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
    try:
        torch.set_num_threads(1)
        out = {}
        for sparse in (True, False):
            g = torch.Generator().manual_seed(100 + rank)
            ps = [torch.zeros(400, 3, requires_grad=True), torch.zeros(400, 1, 15, requires_grad=True),
                  torch.zeros(400, 1, requires_grad=True)]
            bk = GradBucket(ps, rows=row_major)
            assert (bk.rows is not None) == row_major
            rows = torch.randperm(400, generator=g)[: 30 + 20 * rank]  # each rank: its own live rows
            for p in ps:
                p.grad[rows] = torch.randn(p.grad[rows].shape, generator=g)
            bk.allreduce(sparse=sparse)
            out[sparse] = bk.flat.clone().numpy()
        q.put((rank, out[True], out[False]))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("rows", [False, True], ids=["flat", "row_major"])
def test_sparse_bucket_allreduce_equals_dense(rows):
    """GradBucket.allreduce(sparse=True) (union of nonzero rows, packed) == the dense all-reduce, for the flat
    concatenation and for the row-major bucket (one [n, pitch] matrix, each .grad a column block)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sparse_worker, args=(r, 2, port, q, rows)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, sp, de in res:
        np.testing.assert_array_equal(sp, de)
        assert np.count_nonzero(de) > 0
    np.testing.assert_array_equal(res[0][1], res[1][1])


def test_row_major_bucket_layout():
    """GradBucket(rows=True): every parameter's .grad is a column block of one [n, pitch] matrix (4-wide
    parameters first, on 16-B boundaries; pitch a multiple of 16 floats), its shape the parameter's; writes
    through .grad land in the right rows and columns; zero() clears every row; the GaussianModel's six
    tensors (3 + 3 + 45 + 1 + 3 + 4 = 59 floats) get a 64-float pitch with the rotation at column 0."""
    from dge_amd.scene import synthetic_scene

    sc = synthetic_scene(10, sh_degree=3, seed=0).requires_grad_(True)
    bk = GradBucket(sc.parameters(), rows=True)
    assert bk.rows.shape == (10, 64) and bk.check_attached()
    rot = sc._rotation.grad
    assert rot.data_ptr() == bk.rows.data_ptr() and rot.stride() == (64, 1)
    cols = {}
    for name, p in zip(["xyz", "dc", "rest", "op", "sc", "rot"], sc.parameters()):
        assert p.grad.shape == p.shape and p.grad.stride(0) == 64
        cols[name] = (p.grad.data_ptr() - bk.rows.data_ptr()) // 4
        p.grad.fill_(float(len(cols)))
    assert cols["rot"] == 0 and sorted(cols.values()) == [0, 4, 7, 10, 55, 56]
    assert float(bk.rows[:, :59].min()) >= 1.0 and not bk.rows[:, 59:].any()
    assert float(bk.rows[3, 10:55].max()) == 3.0  # (the SH rest block, 45 floats of row 3)
    bk.zero()
    assert not bk.flat.any() and bk.check_attached()


def _order_worker(rank, world, port, pad, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["GLOO_SOCKET_IFNAME"] = "lo"
    os.environ["MASTER_PORT"] = str(port)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
        g = torch.Generator().manual_seed(100 + rank)
        n = 20_000
        # magnitudes over six decades: the 4-term sums' rounding depends on the order of the terms
        v = torch.randn(n, generator=g) * torch.pow(10.0, torch.randint(-3, 3, (n,), generator=g).float())
        dense = v.clone()
        dist.all_reduce(dense)
        shifted = torch.cat([torch.zeros(pad), v])  # the same values at another offset of the buffer
        dist.all_reduce(shifted)
        allv = [torch.empty_like(v) for _ in range(world)]
        dist.all_gather(allv, v)
        q.put((rank, dense.numpy(), shifted[pad:].numpy(), torch.stack(allv).numpy(), None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, None, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _fp32_sums(terms):
    """Every fp32 result of summing the four per-rank terms (columns of `terms` [4, n]) in any order: the
    24 left folds and the 3 x 8 pairwise trees."""
    import itertools

    t = terms.astype(np.float32)
    out = []
    for p in itertools.permutations(range(4)):
        s = t[p[0]]
        for k in p[1:]:
            s = (s + t[k]).astype(np.float32)
        out.append(s)
        out.append(((t[p[0]] + t[p[1]]).astype(np.float32) + (t[p[2]] + t[p[3]]).astype(np.float32)).astype(np.float32))
    return np.stack(out)


@pytest.mark.slow
def test_allreduce_sum_order_depends_on_buffer_position():
    """Why the 4-rank GPU tests compare the packed (sparse-row) all-reduce with the dense one to the rounding of
    the sum and not bit for bit (test_gpu_multiview.py, the deferred union check): gloo's SUM over 4 ranks adds
    an element's 4 terms in an order that depends on where the element sits in the buffer.  The same values
    all-reduced at two offsets of a buffer give different bits for some elements, and every result is one of
    the fp32 sums of the same 4 terms in some order — a reordering of the sum, not an error.  (With 2 ranks
    a + b = b + a: bit for bit.)"""
    world, pad = 4, 1237
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_order_worker, args=(r, world, port, pad, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[4] is None, r[4]
    _, dense, shifted, terms, _ = res[0]
    cand = _fp32_sums(terms)
    assert np.all((cand == dense[None, :]).any(axis=0)), "dense: not a reordering of the 4-term sum"
    assert np.all((cand == shifted[None, :]).any(axis=0)), "shifted: not a reordering of the 4-term sum"
    differ = int((dense != shifted).sum())
    assert differ > 0, "the summation order did not depend on the buffer position"
    for r in res[1:]:  # every rank holds the same result
        np.testing.assert_array_equal(r[1], dense)
        np.testing.assert_array_equal(r[2], shifted)
