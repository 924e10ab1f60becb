"""GPU tests of the multi-view step (SURVEY.md §8(f) F1, configs[2] c3 as far as one card allows):
the 3-view step reductions against the oracle fixture, and the view-sharded step with two ranks
sharing one card (gloo) against the single-process loop."""
from __future__ import annotations

import ctypes
import datetime
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import assert_close

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _Activated:
    """A model whose getters return leaf tensors (the activated values the oracle fixture holds): the
    reference-shaped render() path, gradients land in the leaves."""

    def __init__(self, rec, dev):
        t = lambda k: torch.from_numpy(np.ascontiguousarray(rec[k])).to(dev).requires_grad_(True)
        self.xyz, self.op, self.sh = t("means3D"), t("opacities"), t("shs")
        self.sc, self.rot = t("scales"), t("rotations")
        self.active_sh_degree = self.max_sh_degree = 3
        self.mask = None

    get_xyz = property(lambda self: self.xyz)
    get_opacity = property(lambda self: self.op)
    get_features = property(lambda self: self.sh)
    get_scaling = property(lambda self: self.sc)
    get_rotation = property(lambda self: self.rot)

    def parameters(self):
        return [self.xyz, self.op, self.sh, self.sc, self.rot]

    def num_points(self):
        return int(self.xyz.shape[0])


def test_multiview_step_vs_oracle_3views(cuda_device):
    """multiview_step over 3 views (render + backward per view, gradients summed in the shared bucket):
    radii max identical, the view-space gradient sum within 1e-4 x its terms' magnitude, the summed
    parameter gradients against the oracle's sum (DGE.py:170-296)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import GradBucket, multiview_step

    rec = np.load(os.path.join(GOLDEN, "multiview_3views.npz"))
    dev = torch.device("cuda")
    P, W, H, V = (int(rec[k]) for k in ("P", "W", "H", "V"))
    pc = _Activated(rec, dev)
    cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
    seeds = [torch.from_numpy(rec["dL_dpix"][k]).to(dev) for k in range(V)]
    bucket = GradBucket(pc.parameters())
    out = multiview_step(pc, cams, render, PipelineParams(), torch.zeros(3, device=dev), bucket, V, targets=seeds)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["radii_max"].cpu().numpy(), rec["radii_max"])
    vs = out["viewspace_grad_sum"].cpu().numpy().astype(np.float64)
    err = np.abs(vs[:, :2] - rec["viewspace_grad_sum"][:, :2])
    nbad = int((err > 1e-4 * rec["mag9_sum"][:, :2] + 1e-30).sum())
    print(f"[parity F1] view-space sum elements beyond 1e-4 x magnitude: {nbad}; "
          f"max err/mag {float((err / (rec['mag9_sum'][:, :2] + 1e-30)).max()):.2e}")
    assert nbad == 0 and not vs[:, 2].any()
    for name, p in zip(["means3D", "opacity", "sh", "scales", "rotations"], pc.parameters()):
        assert_close(p.grad.cpu().numpy(), rec[f"dL_d{name}_sum"].reshape(p.shape), f"summed dL_d{name}")
    assert out["found_inf"].item() == 0.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c3_setup(dev, P, V, W, H):
    from dge_amd.cameras import orbit_camera
    from dge_amd.scene import synthetic_scene

    sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
    cams = [orbit_camera(k, 24, W, H, device=dev) for k in range(V)]
    g = torch.Generator().manual_seed(7)
    seeds = [(torch.randn(3, H, W, generator=g) * 1e-3).to(dev) for _ in range(V)]
    return sc, cams, seeds


def _c3_worker(rank, world, port, P, V, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["GLOO_SOCKET_IFNAME"] = "lo"  # (gloo on loopback: the host name need not resolve)
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
        from dge_amd.gaussian_renderer import PipelineParams, render
        from dge_amd.multiview import GradBucket, multiview_step, shard_views

        sc, cams, seeds = _c3_setup(dev, P, V, W, H)
        mine = list(shard_views(V, world, rank))
        bucket = GradBucket(sc.parameters())
        out = multiview_step(sc, [cams[i] for i in mine], render, PipelineParams(), torch.zeros(3, device=dev),
                             bucket, V, targets=[seeds[i] for i in mine])
        torch.cuda.synchronize()
        q.put((rank, bucket.flat.cpu().numpy() if rank == 0 else None, out["viewspace_grad_sum"].cpu().numpy(),
               out["radii_max"].cpu().numpy(), None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, None, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_c3_two_ranks_share_one_card(cuda_device):
    """configs[2]'s per-rank workload (1M Gaussians, the c3 orbit cameras, 3 views per rank) with two
    ranks on one card over gloo: the sparse-row bucket all-reduce, the view-space SUM and radii MAX
    give the single-process 6-view step's results (up to float summation order)."""
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import GradBucket, multiview_step

    P, V, W, H = 1_000_000, 6, 512, 512
    dev = torch.device("cuda", 0)
    sc, cams, seeds = _c3_setup(dev, P, V, W, H)
    bucket = GradBucket(sc.parameters())
    out = multiview_step(sc, cams, render, PipelineParams(), torch.zeros(3, device=dev), bucket, V, targets=seeds)
    torch.cuda.synchronize()
    ref, vs1, r1 = bucket.flat.cpu().numpy(), out["viewspace_grad_sum"].cpu().numpy(), out["radii_max"].cpu().numpy()
    del sc, bucket, out
    torch.cuda.empty_cache()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c3_worker, args=(r, 2, port, P, V, W, H, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, flat, vs, rmax, err in res:
        assert err is None, f"rank {rank}: {err}"
        if flat is not None:
            nz = int(np.count_nonzero(ref))
            print(f"[parity c3x2] bucket nonzero {nz} of {ref.size}; max |d| {float(np.abs(flat - ref).max()):.3e}")
            np.testing.assert_allclose(flat, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
        np.testing.assert_allclose(vs, vs1, rtol=1e-5, atol=1e-6 * np.abs(vs1).max())
        np.testing.assert_array_equal(rmax, r1)
    for p in procs:
        assert p.exitcode == 0


def test_multiview_step_batched_streams_hinted_one_rank(cuda_device):
    """multiview_step(streams=3, bucket_zeroed=True, min_world=1, semantic=True) on a one-rank RCCL group —
    views rendered together on 3 streams, one backward of the summed loss, the all-reduce's live rows agreed
    on before it and the whole protocol run (pack, SUM on the collective's side stream beside the semantic
    renders, unpack) — gives the per-view loop's gradients, view-space sums, radii and semantic masks."""
    import torch.distributed as dist

    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import GradBucket, multiview_step

    dev = torch.device("cuda", 0)
    P, V, W, H = 60_000, 3, 160, 128
    res = {}
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        for mode in ("loop", "batched"):
            sc, cams, seeds = _c3_setup(dev, P, V, W, H)
            bucket = GradBucket(sc.parameters())
            bucket.zero()
            sc.mask = torch.arange(P, device=dev) % 5 == 0  # (the semantic render's colours)
            if mode == "loop":
                out = multiview_step(sc, cams, render, PipelineParams(), torch.zeros(3, device=dev), bucket, V,
                                     targets=seeds, semantic=True)
            else:
                out = multiview_step(sc, cams, render, PipelineParams(), torch.zeros(3, device=dev), bucket, V,
                                     targets=seeds, streams=3, bucket_zeroed=True, min_world=1, semantic=True)
            torch.cuda.synchronize()
            res[mode] = (bucket.flat.clone(), out["viewspace_grad_sum"].clone(), out["radii_max"].clone(),
                         [m.clone() for m in out["semantic_masks"]])
    finally:
        dist.destroy_process_group()
    (g0, v0, r0, m0), (g1, v1, r1, m1) = res["loop"], res["batched"]
    assert len(m0) == V and all(torch.equal(a, b) for a, b in zip(m0, m1)) and any(bool(m.any()) for m in m0)
    assert torch.equal(r0, r1)
    torch.testing.assert_close(v1, v0, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(g1, g0, rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize("V", [1, 3])
@pytest.mark.parametrize("speculate", [False, True])
def test_render_views_batched_matches_per_view_loop(cuda_device, V, speculate):
    """render_views (one autograd node over gs_views_forward / gs_views_backward, the views on V streams)
    against the reference's per-view loop of render() + backward: images, radii, visibility, depth,
    view-space gradients and the accumulated parameter gradients are bitwise equal (the views' per-Gaussian
    passes add into .grad in view order, as the loop's backward calls do); speculate: the binning buffers
    sized from the counts seen before (no host wait), checked afterwards."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import render_views
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    W, H = 320, 256
    cams = [orbit_camera(k, 5, W, H, device=dev) for k in range(V)]
    g = torch.Generator().manual_seed(3)
    seeds = [(torch.randn(3, H, W, generator=g) * 1e-3).to(dev) for _ in range(V)]

    def collect(outs, sc):
        torch.cuda.synchronize()
        res = {f"{k}{i}": o[k].detach().cpu().numpy() for i, o in enumerate(outs)
               for k in ("render", "radii", "visibility_filter", "depth_3dgs")}
        res.update({f"vs{i}": o["viewspace_points"].grad.cpu().numpy() for i, o in enumerate(outs)})
        res.update({f"p{i}": p.grad.cpu().numpy() for i, p in enumerate(sc.parameters())})
        return res

    sc = synthetic_scene(150_000, sh_degree=3, seed=4, device=dev).requires_grad_(True)
    outs = []
    for c, s in zip(cams, seeds):
        o = render(c, sc, PipelineParams(), torch.zeros(3, device=dev))
        o["render"].backward(s)
        outs.append(o)
    ref = collect(outs, sc)  # (the loop's forwards also seed the capacity history)
    for rep in range(2):
        sc = synthetic_scene(150_000, sh_degree=3, seed=4, device=dev).requires_grad_(True)
        outs = render_views(cams, sc, PipelineParams(), torch.zeros(3, device=dev), streams=V, speculate=speculate)
        torch.autograd.backward([o["render"] for o in outs], seeds)
        assert outs.check()
        got = collect(outs, sc)
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} (repeat {rep})")


@pytest.mark.parametrize("merge", ["1", "0", "loop", "side"])
def test_merged_replay_matches_per_view_loop(cuda_device, monkeypatch, merge):
    """Five views on three streams: the backward's replays as ONE launch on the caller's stream per four
    views (k_render_bwd_views: 4 + 1, the views' grids interleaved; DGE_AMD_REPLAY_MERGE=1, the default),
    the same with grids of 8 blocks per view so that every block loops over its items one grid apart
    ("loop": DGE_AMD_REPLAY_GRID_DIV), or one launch per view on the views' streams (=0), then the
    per-Gaussian passes in chunks — every output bitwise the per-view loop's.  "side": three views, the
    merged replay with the live-set pass on a view stream beside it (DGE_AMD_LIVE_SIDE=1)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import render_views
    from dge_amd.scene import synthetic_scene

    monkeypatch.setenv("DGE_AMD_REPLAY_MERGE", "0" if merge == "0" else "1")
    if merge == "loop":
        monkeypatch.setenv("DGE_AMD_REPLAY_GRID_DIV", "1000000")
    monkeypatch.setenv("DGE_AMD_LIVE_SIDE", "1" if merge == "side" else "0")
    dev = torch.device("cuda")
    W, H, V = 288, 224, 3 if merge == "side" else 5
    cams = [orbit_camera(k, 7, W, H, device=dev) for k in range(V)]
    g = torch.Generator().manual_seed(9)
    seeds = [(torch.randn(3, H, W, generator=g) * 1e-3).to(dev) for _ in range(V)]

    def collect(outs, sc):
        torch.cuda.synchronize()
        res = {f"{k}{i}": o[k].detach().cpu().numpy() for i, o in enumerate(outs) for k in ("render", "radii")}
        res.update({f"vs{i}": o["viewspace_points"].grad.cpu().numpy() for i, o in enumerate(outs)})
        res.update({f"p{i}": p.grad.cpu().numpy() for i, p in enumerate(sc.parameters())})
        return res

    sc = synthetic_scene(120_000, sh_degree=3, seed=5, device=dev).requires_grad_(True)
    outs = []
    for c, s in zip(cams, seeds):
        o = render(c, sc, PipelineParams(), torch.zeros(3, device=dev))
        o["render"].backward(s)
        outs.append(o)
    ref = collect(outs, sc)
    sc = synthetic_scene(120_000, sh_degree=3, seed=5, device=dev).requires_grad_(True)
    outs = render_views(cams, sc, PipelineParams(), torch.zeros(3, device=dev), streams=3, speculate=True)
    torch.autograd.backward([o["render"] for o in outs], seeds)
    assert outs.check()
    got = collect(outs, sc)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=f"{k} (merge={merge})")


def test_render_views_speculated_overflow_is_reported(cuda_device):
    """A batch whose instance count outgrows the speculated capacity (the history of this image size holds
    a far smaller scene of the same Gaussian count) is reported by check(); rendered again, it fits and
    equals the exact render."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams
    from dge_amd.multiview import render_views
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    W, H, P = 272, 176, 40_000  # (an image size no other test renders: a fresh count history)
    cams = [orbit_camera(k, 4, W, H, device=dev) for k in range(2)]
    small = synthetic_scene(P, sh_degree=1, seed=2, scale=0.002, device=dev)
    big = synthetic_scene(P, sh_degree=1, seed=2, scale=0.08, device=dev)
    bg = torch.zeros(3, device=dev)
    with torch.no_grad():
        assert render_views(cams, small, PipelineParams(), bg, streams=2).check()  # exact: seeds the history
        spec = render_views(cams, big, PipelineParams(), bg, streams=2, speculate=True)
        assert not spec.check(), "the overflow must be reported"
        again = render_views(cams, big, PipelineParams(), bg, streams=2, speculate=True)
        assert again.check()
        ref = render_views(cams, big, PipelineParams(), bg, streams=2)
        assert ref.check()
    torch.cuda.synchronize()
    assert again.batch.num_rendered == ref.batch.num_rendered
    for o, r in zip(again, ref):
        for k in ("render", "radii", "depth_3dgs"):
            assert torch.equal(o[k], r[k]), k


@pytest.mark.parametrize("W,H,P", [(320, 256, 120_000), (1920, 1080, 300_000)])
def test_forward_only_renders_equal_training_renders(cuda_device, W, H, P):
    """Renders under no_grad (or of a scene without gradients) set gs_params.forward_only: the kernels skip
    the backward's scratch (checkpoints, binning flags, per-Gaussian work lists) and the blend's backward
    bookkeeping; on grids over 2048 tiles (1080p: the two-level binning) their lists also carry the Gaussian
    ids alone (no binning slots).  Image, depth, radii and the instance count equal the training render's,
    for render() and the batched render_views."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import render_views
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    cams = [orbit_camera(k, 3, W, H, device=dev) for k in range(3)]
    bg = torch.tensor([0.1, 0.2, 0.3], device=dev)
    sc = synthetic_scene(P, sh_degree=3, seed=6, device=dev).requires_grad_(True)
    train = [render(c, sc, PipelineParams(), bg) for c in cams]
    train_views = render_views(cams, sc, PipelineParams(), bg, streams=3)
    with torch.no_grad():
        fwd = [render(c, sc, PipelineParams(), bg) for c in cams]
        fwd_views = render_views(cams, sc, PipelineParams(), bg, streams=3)
        colors = torch.rand(sc.num_points(), 3, generator=torch.Generator().manual_seed(1)).to(dev)
        sem = [render(c, sc, PipelineParams(), bg, override_color=colors) for c in cams]
    sem_train = [render(c, sc, PipelineParams(), bg, override_color=colors.requires_grad_(True)) for c in cams]
    assert fwd_views.check() and train_views.check()
    torch.cuda.synchronize()
    for pairs in ((train, fwd), (train_views, fwd_views), (train, fwd_views), (sem_train, sem)):
        for a, b in zip(*pairs):
            for k in ("render", "radii", "depth_3dgs"):
                assert torch.equal(a[k].detach(), b[k]), k
    assert train_views.batch.num_rendered == fwd_views.batch.num_rendered


def _hinted_worker(rank, world, port, P, V, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["GLOO_SOCKET_IFNAME"] = "lo"  # (gloo on loopback: the host name need not resolve)
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
        from dge_amd.gaussian_renderer import PipelineParams, render
        from dge_amd.multiview import GradBucket, multiview_step, shard_views

        sc, cams, seeds = _c3_setup(dev, P, V, W, H)
        sc.mask = torch.arange(P, device=dev) % 5 == 0
        mine = list(shard_views(V, world, rank))
        bucket = GradBucket(sc.parameters())
        bucket.zero()
        out = multiview_step(sc, [cams[i] for i in mine], render, PipelineParams(), torch.zeros(3, device=dev),
                             bucket, V, targets=[seeds[i] for i in mine], streams=3, bucket_zeroed=True,
                             semantic=True)
        torch.cuda.synchronize()
        # this rank's own rows: the Gaussians its views blend (the rows only this rank touches must arrive)
        q.put((rank, bucket.flat.cpu().numpy(), [m.cpu().numpy() for m in out["semantic_masks"]], None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_hinted_sparse_allreduce_two_ranks(cuda_device):
    """The agreed-before-backward sparse all-reduce (GradBucket.allreduce_begin/_end, the collective on a
    side stream beside the semantic renders) with two ranks on one card (gloo, CUDA tensors), 2 views
    each: both ranks hold the single-process 4-view step's summed gradients — including rows only one
    rank's views touch — and each rank's semantic masks are its views' masks in the single-process step."""
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import GradBucket, multiview_step

    P, V, W, H = 60_000, 4, 160, 128
    dev = torch.device("cuda", 0)
    sc, cams, seeds = _c3_setup(dev, P, V, W, H)
    sc.mask = torch.arange(P, device=dev) % 5 == 0
    bucket = GradBucket(sc.parameters())
    out = multiview_step(sc, cams, render, PipelineParams(), torch.zeros(3, device=dev), bucket, V, targets=seeds,
                         semantic=True)
    torch.cuda.synchronize()
    ref = bucket.flat.cpu().numpy()
    masks = [m.cpu().numpy() for m in out["semantic_masks"]]
    # each rank's own contribution (its two views alone): the elements only one rank's views make nonzero
    half = []
    for idx in ((0, 1), (2, 3)):
        b2 = GradBucket(sc.parameters())
        multiview_step(sc, [cams[i] for i in idx], render, PipelineParams(), torch.zeros(3, device=dev), b2, V,
                       targets=[seeds[i] for i in idx])
        torch.cuda.synchronize()
        half.append(b2.flat.cpu().numpy())
        del b2
    del sc, bucket, out
    torch.cuda.empty_cache()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hinted_worker, args=(r, 2, port, P, V, W, H, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    only0 = (half[0] != 0) & (half[1] == 0)
    only1 = (half[1] != 0) & (half[0] == 0)
    assert only0.any() and only1.any()
    for rank, flat, sems, err in res:
        assert err is None, f"rank {rank}: {err}"
        np.testing.assert_allclose(flat, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
        assert np.array_equal(flat[only0] != 0, ref[only0] != 0) and np.array_equal(flat[only1] != 0, ref[only1] != 0)
        mine = (0, 1) if rank == 0 else (2, 3)
        assert all(np.array_equal(a, masks[i]) for a, i in zip(sems, mine))
    for p in procs:
        assert p.exitcode == 0


def test_zeroed_bucket_stores_first_gradient(cuda_device):
    """GradBucket.zero() registers the cleared buffer, and the next batched backward into it stores each
    Gaussian's first gradient instead of adding it to the zeros (gs_grads.zeroed: no read of the zeros).
    The bucket equals the read-modify-write path's (registration dropped) bit for bit, and the registration
    is taken by that backward: a second backward without a zero adds (twice the first sums, up to the
    order of the additions)."""
    from dge_amd import diff_gaussian_rasterization as R
    from dge_amd.gaussian_renderer import PipelineParams
    from dge_amd.multiview import GradBucket, render_views

    dev = torch.device("cuda", 0)
    P, V, W, H = 60_000, 3, 160, 128
    sc, cams, seeds = _c3_setup(dev, P, V, W, H)
    bucket = GradBucket(sc.parameters())
    bg = torch.zeros(3, device=dev)

    def step():
        outs = render_views(cams, sc, PipelineParams(), bg, streams=3)
        torch.autograd.backward([o["render"] for o in outs], seeds)
        torch.cuda.synchronize()

    res = {}
    for mode in ("add", "store"):
        bucket.zero()
        if mode == "add":
            R._ZEROED.clear()
        else:
            assert dev.index in R._ZEROED
        step()
        assert dev.index not in R._ZEROED
        res[mode] = bucket.flat.clone()
    assert torch.equal(res["store"], res["add"]) and bool(res["store"].abs().sum() > 0)
    step()  # no zero in between: adds
    # (a store would leave the first sums: half of these; the views' terms cancel in a few elements)
    torch.testing.assert_close(bucket.flat, 2 * res["store"], rtol=1e-5, atol=1e-6 * float(res["store"].abs().max()))


def _deferred_worker(rank, world, port, P, V, W, H, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["GLOO_SOCKET_IFNAME"] = "lo"  # (gloo on loopback: the host name need not resolve)
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
        from dge_amd.gaussian_renderer import PipelineParams
        from dge_amd.multiview import GradBucket, render_views, shard_views

        sc, cams, seeds = _c3_setup(dev, P, V, W, H)
        mine = list(shard_views(V, world, rank))
        bucket = GradBucket(sc.parameters())
        bg = torch.zeros(3, device=dev)
        errs = []
        # step 0 sets the speculated capacity; step 1 runs under it, step 2 under a third of the union (the
        # deferred check finds the overflow and all-reduces the rows past the capacity)
        for k, cap in enumerate((None, None, "third")):
            bucket.zero()
            outs = render_views([cams[i] for i in mine], sc, PipelineParams(), bg, streams=3, speculate=True)
            bucket.allreduce_begin([o["_live_rows"] for o in outs], min_world=2)
            torch.autograd.backward([o["render"] for o in outs], [seeds[i] for i in mine])
            assert outs.check()
            torch.cuda.synchronize()
            dense = bucket.flat.clone()
            dist.all_reduce(dense, op=dist.ReduceOp.SUM)
            if cap == "third":
                bucket._rows_cap = max(1, (bucket._rows_cap - 4096) * 8 // 9 // 3)  # (cap = m + m // 8 + 4096)
            spec = bucket._rows_cap > 0
            bucket.allreduce_end(defer_check=True)
            deferred = getattr(bucket, "_deferred", None) is not None
            fixed = bucket.allreduce_finalize()
            torch.cuda.synchronize()
            # two ranks: a + b in either order, bit for bit; more ranks: RCCL / gloo add the ranks' rows in an
            # order that depends on where the row sits in the buffer (packed or dense), so to the sum's rounding
            same = bool(torch.equal(bucket.flat, dense)) if world == 2 else bool(torch.allclose(
                bucket.flat, dense, rtol=1e-5, atol=1e-6 * float(dense.abs().max())))
            errs.append((k, spec, deferred, fixed, same, int((dense != 0).sum())))
        q.put((rank, errs, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,V", [(2, 4), (4, 10)], ids=["2ranks_4views", "4ranks_10views"])
def test_deferred_union_check_two_ranks(cuda_device, world, V):
    """allreduce_end(defer_check=True) + allreduce_finalize() (the bench's distributed step): with two or
    four ranks on one card (gloo, CUDA tensors; 10 views over 4 ranks: uneven 3/3/2/2 shards), the bucket
    after the packed SUM at a speculated capacity equals the dense all-reduce of the ranks' buckets (bit for
    bit with two ranks; with four, to the rounding of the collective's rank order, which depends on the
    row's position in the buffer: shown on the CPU by test_allreduce_sum_order_depends_on_buffer_position,
    where every 4-rank result is an fp32 reordering of the same sum) — also when the capacity is a third of
    the union and the deferred check all-reduces the rows past it."""
    P, W, H = 300_000, 160, 128  # (a union under half the rows: the packed path)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_deferred_worker, args=(r, world, port, P, V, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, steps, err in res:
        assert err is None, f"rank {rank}: {err}"
        print(f"[deferred] rank {rank}: (step, speculated, deferred, fix-up, equal, nonzero) {steps}")
        (k0, s0, d0, f0, e0, _), (k1, s1, d1, f1, e1, _), (k2, s2, d2, f2, e2, _) = steps
        assert not s0 and not d0 and e0          # first step: exact (no capacity yet)
        assert s1 and d1 and not f1 and e1       # speculated, deferred, no overflow
        assert s2 and d2 and f2 and e2           # capacity below the union: the deferred fix-up ran


def _seed_history(dev, P, cams, sc, small):
    """Render `cams` exactly once (no gradients) to seed this process's speculated-capacity history for
    their (P, W, H): with the scene itself, or (small) with the same number of Gaussians moved out of
    every frustum — a capacity of 64k instances, far below the scene's count."""
    from dge_amd.gaussian_renderer import PipelineParams
    from dge_amd.multiview import render_views
    from dge_amd.scene import synthetic_scene

    if small:
        sc = synthetic_scene(P, seed=1, device=dev)
        sc._xyz += 1000.0
    with torch.no_grad():
        assert render_views(cams, sc, PipelineParams(), torch.zeros(3, device=dev), streams=3).check()


def _overflow_worker(rank, world, port, P, V, sizes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["GLOO_SOCKET_IFNAME"] = "lo"  # (gloo on loopback: the host name need not resolve)
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=90))
        from dge_amd.gaussian_renderer import PipelineParams, render
        from dge_amd.multiview import GradBucket, multiview_step, render_views, shard_views

        mine = list(shard_views(V, world, rank))
        bg = torch.zeros(3, device=dev)
        out = {}
        # (1) multiview_step (hinted, the check inside allreduce_end) at sizes[0]; (2) the bench's step —
        # a speculated packed SUM whose union check is deferred — at sizes[2], after a first step at
        # sizes[1] that sets the packed capacity.  Only rank 1's history is seeded with the small scene.
        W, H = sizes[0]
        sc, cams, seeds = _c3_setup(dev, P, V, W, H)
        _seed_history(dev, P, [cams[i] for i in mine], sc, small=rank == 1)
        bucket = GradBucket(sc.parameters())
        bucket.zero()
        multiview_step(sc, [cams[i] for i in mine], render, PipelineParams(), bg, bucket, V,
                       targets=[seeds[i] for i in mine], streams=3, bucket_zeroed=True)
        torch.cuda.synchronize()
        out["step"] = bucket.flat.cpu().numpy()
        del bucket
        for k, (W, H) in enumerate(sizes[1:]):
            sc, cams, seeds = _c3_setup(dev, P, V, W, H)
            if k == 0:
                bucket = GradBucket(sc.parameters())
            else:
                bucket.params = sc.parameters()
                _seed_history(dev, P, [cams[i] for i in mine], sc, small=rank == 1)
            bucket.zero()
            retried = False
            outs = render_views([cams[i] for i in mine], sc, PipelineParams(), bg, streams=3, speculate=True)
            bucket.allreduce_begin([o["_live_rows"] for o in outs], views=outs)
            torch.autograd.backward([o["render"] for o in outs], [seeds[i] for i in mine])
            if not outs.check():
                retried = True
                bucket.zero()
                outs = render_views([cams[i] for i in mine], sc, PipelineParams(), bg, streams=3, speculate=True)
                torch.autograd.backward([o["render"] for o in outs], [seeds[i] for i in mine])
                assert outs.check()
            spec = bucket._rows_cap > 0
            bucket.allreduce_end(defer_check=True)
            deferred = getattr(bucket, "_deferred", None) is not None
            fixed = bucket.allreduce_finalize()
            torch.cuda.synchronize()
            out[f"deferred{k}"] = (bucket.flat.cpu().numpy() if k else None, retried, spec, deferred, fixed)
        q.put((rank, out, None))
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((rank, None, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,V", [(2, 4), (4, 10)], ids=["2ranks_4views", "4ranks_10views"])
def test_overflow_on_one_rank_is_agreed(cuda_device, world, V):
    """A speculated batch that overflows its binning capacity on ONE rank only (rank 1: its capacity
    history holds a scene with no visible Gaussian): the overflowing rank re-renders locally, the overflow
    flag rides the union's MAX collective, and every rank runs the same collectives — no hang, no
    mismatched reduction — ending with the single-process step's summed gradients, in multiview_step and
    in the bench's deferred-check step.  Two or four ranks on one card (gloo, CUDA tensors); 10 views over
    4 ranks is the uneven 3/3/2/2 sharding, rank 1 a non-last rank."""
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import GradBucket, multiview_step

    P = 300_000
    sizes = [(176, 128), (160, 128), (192, 128)]
    dev = torch.device("cuda", 0)
    refs = {}
    for key, (W, H) in (("step", sizes[0]), ("deferred1", sizes[2])):
        sc, cams, seeds = _c3_setup(dev, P, V, W, H)
        bucket = GradBucket(sc.parameters())
        multiview_step(sc, cams, render, PipelineParams(), torch.zeros(3, device=dev), bucket, V, targets=seeds)
        torch.cuda.synchronize()
        refs[key] = bucket.flat.cpu().numpy()
        del sc, bucket
    torch.cuda.empty_cache()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_overflow_worker, args=(r, world, port, P, V, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=150) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, out, err in res:
        assert err is None, f"rank {rank}: {err}"
        ref = refs["step"]
        np.testing.assert_allclose(out["step"], ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
        _, r0, s0, d0, f0 = out["deferred0"]
        flat, r1, s1, d1, f1 = out["deferred1"]
        print(f"[overflow] rank {rank}: first step (retried, spec, deferred, fix-up) {(r0, s0, d0, f0)}, "
              f"overflow step {(r1, s1, d1, f1)}")
        assert not r0
        assert r1 == (rank == 1), "only rank 1's capacity is too small"
        assert s1 and d1 and f1, "the agreed flag must turn the deferred check into the scanning all-reduce"
        ref = refs["deferred1"]
        np.testing.assert_allclose(flat, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
    for p in procs:
        assert p.exitcode == 0


def _c2_bench_setup(dev, P=1_000_000, W=512, H=512, V=3):
    """bench.py's c2 workload: the seeded 1M scene, the 3 orbit views of a one-rank run, its seeds."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.scene import synthetic_scene

    sc = synthetic_scene(P, sh_degree=3, seed=0, device=dev).requires_grad_(True)
    cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
    gen = torch.Generator(device="cpu").manual_seed(1)
    seeds = [(torch.randn(3, H, W, generator=gen) * 1e-3).to(dev) for _ in range(V)]
    return sc, cams, seeds


def test_c2_timed_path_matches_per_view_loop(cuda_device, oracle):
    """The path bench.py times, at the timed size (c2: 1M Gaussians, 512x512, 3 orbit views): render_views
    on 3 streams with speculated binning capacities (capacity-sized tile-sort grids, the count read on the
    device), the bucket zeroed on a view stream beside the forwards (GradBucket.zero(stream=...): the
    backward stores each Gaussian's first gradient), one backward of the summed loss — against the
    reference's per-view loop of render() + backward (exact binning: the host waits for each count,
    rasterizer_impl.cu:236-270): images, depths, radii, view-space gradients and the whole gradient bucket
    bit for bit, twice; view 0's forward bit-identical to the oracle's (lists, ranges, n_contrib, T)."""
    from dge_amd import _native as N
    from dge_amd.gaussian_renderer import PipelineParams, _settings, render
    from dge_amd.multiview import GradBucket, render_views, view_streams
    from helpers import compare_forward, run_oracle, views_forward_dict

    dev = torch.device("cuda", 0)
    P, W, H, V = 1_000_000, 512, 512, 3
    sc, cams, seeds = _c2_bench_setup(dev, P, W, H, V)
    bg = torch.zeros(3, device=dev)
    bucket = GradBucket(sc.parameters())
    bucket.zero()
    ref_outs = []
    for c, s in zip(cams, seeds):  # (also seeds the capacity history of this (P, W, H))
        o = render(c, sc, PipelineParams(), bg)
        o["render"].backward(s)
        ref_outs.append(o)
    torch.cuda.synchronize()
    keys = ("render", "depth_3dgs", "radii", "visibility_filter")
    ref = {f"{k}{v}": o[k].detach().clone() for v, o in enumerate(ref_outs) for k in keys}
    ref.update({f"vs{v}": o["viewspace_points"].grad.clone() for v, o in enumerate(ref_outs)})
    ref["bucket"] = bucket.flat.clone()
    del ref_outs
    for rep in range(2):
        outs = render_views(cams, sc, PipelineParams(), bg, streams=3, speculate=True)
        bucket.zero(stream=view_streams(dev, 3)[1])  # (as bench.py: the view stream waits for the fork)
        torch.autograd.backward([o["render"] for o in outs], seeds)
        assert outs.check()
        torch.cuda.synchronize()
        layout = [int(N.lib().gs_views_layout(outs.batch.handle, v)) for v in range(V)]
        print(f"[c2 timed path] rep {rep}: num_rendered {outs.batch.num_rendered}, capacity {layout}")
        assert all(0 < k < c for k, c in zip(outs.batch.num_rendered, layout)), "speculated, capacity-sized"
        got = {f"{k}{v}": o[k].detach() for v, o in enumerate(outs) for k in keys}
        got.update({f"vs{v}": o["viewspace_points"].grad for v, o in enumerate(outs)})
        got["bucket"] = bucket.flat
        for k in ref:
            assert torch.equal(got[k], ref[k]), f"{k} (repeat {rep})"
    assert bool(ref["bucket"].abs().sum() > 0)
    # view 0 of the last batch against the oracle (its speculated binning, read at the capacity layout)
    fwd = views_forward_dict(outs.batch, 0, outs[0]["render"], outs[0]["depth_3dgs"], outs[0]["radii"])
    with torch.no_grad():
        # the oracle takes activated parameters; the kernels activate the raw ones in-kernel (sigmoid /
        # exp / normalize on the device's libm, which differ from torch's in the last bit for a third of
        # the rows): the oracle gets the device's activations (gs_activate_params: the preprocess's own
        # device functions)
        op = torch.empty(P, 1, device=dev)
        scl = torch.empty(P, 3, device=dev)
        rot = torch.empty(P, 4, device=dev)
        N.check(N.lib().gs_activate_params(P, sc._opacity.data_ptr(), sc._scaling.data_ptr(), sc._rotation.data_ptr(),
                                           op.data_ptr(), scl.data_ptr(), rot.data_ptr(),
                                           ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                "gs_activate_params")
        kw = dict(means3D=sc.get_xyz.cpu().numpy(), opacities=op.cpu().numpy(),
                  shs=sc.get_features.cpu().numpy(), scales=scl.cpu().numpy(), rotations=rot.cpu().numpy())
    from dge_amd.cameras import orbit_camera

    rs = _settings(orbit_camera(0, V, W, H, device="cpu"), torch.zeros(3), 1.0, 3)
    compare_forward(fwd, run_oracle(oracle, rs, **kw), label="c2 timed path, view 0")


def test_c2_speculated_overflow_at_full_size(cuda_device):
    """A forced overflow at c2 size: the capacity history of this (P, W, H) holds a scene of the same
    Gaussian count with none in view (a 64k-instance capacity against ~3.6M instances).  check() reports
    it; the batch rendered again fits and equals the exact render (images, depths, radii, num_rendered)
    and its backward equals the exact batch's bucket, bit for bit."""
    from dge_amd.gaussian_renderer import PipelineParams
    from dge_amd.multiview import GradBucket, render_views
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda", 0)
    P, W, H, V = 1_000_003, 512, 512, 3  # (a Gaussian count no other test renders: a fresh history)
    sc, cams, seeds = _c2_bench_setup(dev, P, W, H, V)
    bg = torch.zeros(3, device=dev)
    far = synthetic_scene(P, sh_degree=3, seed=1, device=dev)
    far._xyz += 1000.0
    with torch.no_grad():
        first = render_views(cams, far, PipelineParams(), bg, streams=3)
        assert first.check() and max(first.batch.num_rendered) == 0
    del far
    bucket = GradBucket(sc.parameters())
    res = {}
    for mode in ("spec", "exact"):
        bucket.zero()
        outs = render_views(cams, sc, PipelineParams(), bg, streams=3, speculate=mode == "spec")
        if mode == "spec":
            torch.autograd.backward([o["render"] for o in outs], seeds)
            assert not outs.check(), "the overflow must be reported"
            print(f"[c2 overflow] reported: num_rendered {outs.batch.num_rendered}")
            bucket.zero()
            outs = render_views(cams, sc, PipelineParams(), bg, streams=3, speculate=True)
        torch.autograd.backward([o["render"] for o in outs], seeds)
        assert outs.check()
        torch.cuda.synchronize()
        res[mode] = ([{k: o[k].detach().clone() for k in ("render", "depth_3dgs", "radii")} for o in outs],
                     list(outs.batch.num_rendered), bucket.flat.clone())
    (a, ka, ga), (b, kb, gb) = res["spec"], res["exact"]
    assert ka == kb and min(ka) > 1_000_000
    for x, y in zip(a, b):
        for k in x:
            assert torch.equal(x[k], y[k]), k
    assert torch.equal(ga, gb)


def test_lazy_override_color_render(cuda_device, monkeypatch):
    """DGE's semantic render (render(..., override_color=mask colours) with grad mode on, DGE.py:198-204)
    runs the forward-only kernels; its image, depth and radii equal the eager training render's, and a
    backward through it (which DGE never runs) recomputes the forward with the backward's bookkeeping and
    gives the eager render's gradients bit for bit — also a second backward (retain_graph)."""
    from dge_amd import gaussian_renderer as GR
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda", 0)
    W, H = 256, 192
    cam = orbit_camera(1, 4, W, H, device=dev)
    G = torch.randn(3, H, W, generator=torch.Generator().manual_seed(4)).to(dev)
    colors = torch.rand(50_000, 3, generator=torch.Generator().manual_seed(5)).to(dev)
    res = {}
    for lazy in (True, False):
        monkeypatch.setattr(GR, "_LAZY_OVERRIDE", lazy)
        sc = synthetic_scene(50_000, seed=9, device=dev).requires_grad_(True)
        pkg = render(cam, sc, PipelineParams(), torch.zeros(3, device=dev), override_color=colors)
        out = [pkg[k].detach().clone() for k in ("render", "depth_3dgs", "radii")]
        (pkg["render"] * G).sum().backward(retain_graph=True)
        g1 = [p.grad.clone() for p in (sc._xyz, sc._opacity, sc._scaling, sc._rotation)]
        (pkg["render"] * G).sum().backward()
        g2 = [p.grad.clone() for p in (sc._xyz, sc._opacity, sc._scaling, sc._rotation)]
        torch.cuda.synchronize()
        res[lazy] = (out, g1, g2, pkg["viewspace_points"].grad.clone())
    (oa, ga1, ga2, va), (ob, gb1, gb2, vb) = res[True], res[False]
    for x, y in zip(oa, ob):
        assert torch.equal(x, y)
    assert torch.equal(va, vb) and bool(va.abs().sum() > 0)
    for x, y in zip(ga1 + ga2, gb1 + gb2):
        assert torch.equal(x, y)


def test_views_backward_after_outputs_dropped(cuda_device):
    """The batch keeps what its backward reads: a caller that keeps only the images (DGE's loop drops a
    view's dict once it has taken the radii max) and allocates in between gets the same gradients, bit for
    bit, as one that keeps every output (the radii block was once handed to other tensors meanwhile)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams
    from dge_amd.multiview import render_views
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, W, H = 40_000, 176, 144
    cams = [orbit_camera(k, 4, W, H, device=dev) for k in range(3)]
    Gs = [torch.randn(3, H, W, generator=torch.Generator().manual_seed(60 + k)).to(dev) for k in range(3)]

    def run(keep):
        sc = synthetic_scene(P, seed=21, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
        outs = render_views(cams, sc, PipelineParams(), torch.zeros(3, device=dev), streams=3, speculate=True)
        assert outs.check()
        imgs = [o["render"] for o in outs]
        if not keep:
            del outs
            junk = [torch.full((len(cams), P), -7, dtype=torch.int32, device=dev) for _ in range(4)]
            del junk
        torch.autograd.backward(imgs, Gs)
        torch.cuda.synchronize()
        return [p.grad.clone() for p in sc.parameters()]

    ref = run(True)
    got = run(False)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), f"parameter {i}"
