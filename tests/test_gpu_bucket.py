"""GPU tests of the sparse-row gradient exchange kernels (gs_rows_live / gs_rows_gather /
gs_rows_scatter and their device-count forms, dge_amd/csrc/gs_bucket.hip) against the torch formulation GradBucket uses on CPU:
bit-exact (pure data movement and a != 0 test)."""
import pytest
import torch

from dge_amd import multiview as mv

pytestmark = pytest.mark.gpu


def _mats(n, widths, density, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    flat = torch.zeros(n * sum(widths))
    mats, off = [], 0
    for w in widths:
        m = flat[off:off + n * w].view(n, w)
        rows = torch.rand(n, generator=g) < density
        m[rows] = torch.randn(int(rows.sum()), w, generator=g)
        # a live row may hold a single nonzero in any column; -0.0 is zero, NaN is not
        pick = torch.randint(0, w, (n,), generator=g)
        lone = (torch.rand(n, generator=g) < density) & ~rows
        m[lone.nonzero().squeeze(1), pick[lone]] = 1.0
        mats.append(m)
        off += n * w
    mats[0][1, 0] = -0.0
    mats[-1][2, -1] = float("nan")
    flat = flat.to(device)
    out, off = [], 0
    for w in widths:
        out.append(flat[off:off + n * w].view(n, w))
        off += n * w
    return flat, out


@pytest.mark.parametrize("n,widths,density", [(1_000_003, (3, 3, 45, 1, 3, 4), 0.1), (300, (1,), 0.5),
                                              (5000, (7, 2), 0.0), (4096, (64,), 1.0)])
def test_rows_live_gather_scatter_match_torch(cuda_device, n, widths, density):
    flat, mats = _mats(n, widths, density, seed=n, device="cuda")
    assert mv._native_ok(mats)
    live = mv._rows_live(mats, n)
    ref = torch.zeros(n, dtype=torch.uint8)
    for m in mats:
        ref |= (m.cpu() != 0).any(1).to(torch.uint8)
    assert torch.equal(live.cpu(), ref)
    idx = torch.nonzero(live).squeeze(1)
    packed = mv._rows_gather(mats, idx)
    ref_packed = torch.cat([m.cpu().index_select(0, idx.cpu()) for m in mats], 1)
    assert torch.equal(packed.cpu().view(torch.int32), ref_packed.view(torch.int32))
    # scatter back doubled values into a zeroed copy: rows outside idx stay zero
    flat2, mats2 = torch.zeros_like(flat), []
    off = 0
    for w in widths:
        mats2.append(flat2[off:off + n * w].view(n, w))
        off += n * w
    mv._rows_scatter(mats2, idx, packed * 2)
    torch.cuda.synchronize()
    for m, m2 in zip(mats, mats2):
        exp = torch.zeros(n, m.shape[1])
        exp[idx.cpu()] = m.cpu()[idx.cpu()] * 2
        assert torch.equal(m2.cpu().nan_to_num(7.0), exp.nan_to_num(7.0))


@pytest.mark.parametrize("n,width,pitch", [(1_000_003, 59, 64), (257, 1, 3), (4099, 13, 16)])
def test_rows_pitched_region_ignores_padding(cuda_device, n, width, pitch):
    """A region that is the first `width` columns of `pitch`-float rows (GradBucket.row_matrices: the 59 used
    columns of a GaussianModel's 64-float bucket row, ABI 21): live marks only rows nonzero in those columns
    (the padding holds nonzeros here), the gather packs `width` columns, the scatter leaves the padding."""
    g = torch.Generator(device="cpu").manual_seed(n)
    full = torch.zeros(n, pitch)
    rows = torch.rand(n, generator=g) < 0.2
    full[rows, :width] = torch.randn(int(rows.sum()), width, generator=g)
    full[:, width:] = 5.0  # padding: never a live mark, never moved
    full = full.to("cuda")
    m = full[:, :width]
    assert mv._native_ok([m]) and not m.is_contiguous()
    live = mv._rows_live([m], n)
    assert torch.equal(live.cpu(), rows.to(torch.uint8))
    idx = torch.nonzero(live).squeeze(1)
    packed = mv._rows_gather([m], idx)
    assert packed.shape == (idx.numel(), width)
    assert torch.equal(packed.cpu(), full.cpu()[idx.cpu(), :width])
    full2 = torch.full_like(full, 9.0)
    mv._rows_scatter([full2[:, :width]], idx, packed * 2)
    torch.cuda.synchronize()
    exp = torch.full((n, pitch), 9.0)
    exp[idx.cpu(), :width] = full.cpu()[idx.cpu(), :width] * 2
    assert torch.equal(full2.cpu(), exp)


@pytest.mark.parametrize("cap_over", [-1000, 0, 1, 5000, None])
def test_rows_gather_scatter_device_count(cuda_device, cap_over):
    """gs_rows_gather_dev / gs_rows_scatter_dev (the speculative-capacity collective): a packed buffer of
    `cap` rows from a row list whose count is read on the device — rows past min(cap, count) packed as
    zeros, the scatter writing back only the first min(cap, count) rows."""
    n, widths = 200_003, (3, 45, 1, 4)
    flat, mats = _mats(n, widths, 0.2, seed=11, device="cuda")
    idx = torch.nonzero(mv._rows_live(mats, n)).squeeze(1)
    m = idx.numel()
    count = m if cap_over is not None else 0
    cap = max(1, m + (cap_over or 0))
    idx_pad = torch.cat([idx, torch.full((max(0, cap - m) + 7,), -5, dtype=torch.int64, device="cuda")])
    cnt = torch.tensor([count], dtype=torch.int64, device="cuda")
    packed = mv._rows_gather(mats, idx_pad, cap=cap, count=cnt)
    k = min(cap, count)
    ref = torch.zeros(cap, sum(widths))
    ref[:k] = torch.cat([mm.cpu().index_select(0, idx[:k].cpu()) for mm in mats], 1)
    assert torch.equal(packed.cpu().view(torch.int32), ref.view(torch.int32))
    flat2 = torch.zeros_like(flat)
    mats2, off = [], 0
    for w in widths:
        mats2.append(flat2[off:off + n * w].view(n, w))
        off += n * w
    mv._rows_scatter(mats2, idx_pad, packed + 1.0, cap=cap, count=cnt)
    torch.cuda.synchronize()
    for mm, m2 in zip(mats, mats2):
        exp = torch.zeros(n, mm.shape[1])
        exp[idx[:k].cpu()] = mm.cpu()[idx[:k].cpu()] + 1.0
        assert torch.equal(m2.cpu().nan_to_num(7.0), exp.nan_to_num(7.0))


@pytest.mark.parametrize("n,density", [(1_000_003, 0.1), (1, 1.0), (2047, 0.0), (4096, 1.0), (70_000, 0.5),
                                       (3_100_000, 0.3)])  # (the last: blocks of several 1024-row runs)
def test_rows_compact_matches_nonzero(cuda_device, n, density):
    """gs_rows_compact: the ascending live rows and their count, no host round trip (vs torch.nonzero)."""
    from dge_amd import _native as N

    g = torch.Generator(device="cpu").manual_seed(n)
    live = ((torch.rand(n, generator=g) < density).to(torch.uint8) * torch.randint(1, 255, (n,), generator=g,
                                                                                     dtype=torch.uint8)).cuda()
    rows = torch.full((n,), -7, dtype=torch.int64, device="cuda")
    cs = torch.empty(1 + (n + 1023) // 1024, dtype=torch.int64, device="cuda")
    N.check(N.lib().gs_rows_compact(live.data_ptr(), n, rows.data_ptr(), cs.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream), "gs_rows_compact")
    ref = torch.nonzero(live).squeeze(1)
    m = int(cs[0].item())
    assert m == ref.numel()
    assert torch.equal(rows[:m], ref)


def test_allreduce_begin_end_one_rank(cuda_device):
    """The hinted protocol on a one-rank RCCL group (the bench's multi-GPU step): the forwards' blended
    Gaussians cover every nonzero gradient row, and the packed SUM leaves the bucket unchanged (one rank);
    the union it agreed on equals the rows the bucket scan finds nonzero."""
    import os

    import torch.distributed as dist

    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams
    from dge_amd.scene import synthetic_scene

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda_device)
    try:
        sc = synthetic_scene(50_000, seed=9, device=cuda_device).requires_grad_(True)
        cams = [orbit_camera(k, 3, 192, 160, device=cuda_device) for k in range(3)]
        G = [torch.randn(3, 160, 192, generator=torch.Generator().manual_seed(k)).to(cuda_device) for k in range(3)]
        bucket = mv.GradBucket(sc.parameters())
        bucket.flat.fill_(3.0)
        outs = mv.render_views(cams, sc, PipelineParams(), torch.zeros(3, device=cuda_device), streams=3)
        bucket.zero(overlap=True)
        hints = [o["_live_rows"] for o in outs]
        bucket.allreduce_begin(hints, min_world=1)
        assert bucket._pending[0] == "hint"
        torch.autograd.backward([o["render"] for o in outs], G)
        torch.cuda.synchronize()
        before = bucket.flat.clone()
        n = sc._xyz.shape[0]
        mats = bucket.row_matrices()
        nonzero = mv._rows_live(mats, n).bool()
        union = torch.zeros(n, dtype=torch.bool, device=cuda_device)
        for h in hints:
            union |= h.bool()
        assert not (nonzero & ~union).any()  # every nonzero gradient row is in the agreed union
        assert torch.equal(union, nonzero)   # ... and the union is exactly the backward's live set
        bucket.allreduce_end()
        torch.cuda.synchronize()
        assert torch.equal(bucket.flat, before)
        m = int(union.sum())
        assert bucket._rows_cap > m  # the next step's speculative capacity
        # later steps: the packed SUM at a speculative capacity (above the union, then below it: the
        # rows past the capacity follow in the exact fix-up collective) leaves the bucket unchanged too
        for cap in (bucket._rows_cap, m // 3):
            bucket.zero(overlap=True)
            outs = mv.render_views(cams, sc, PipelineParams(), torch.zeros(3, device=cuda_device), streams=3)
            bucket.allreduce_begin([o["_live_rows"] for o in outs], min_world=1)
            torch.autograd.backward([o["render"] for o in outs], G)
            bucket._rows_cap = cap
            torch.cuda.synchronize()
            before = bucket.flat.clone()
            assert int((mv._rows_live(mats, n) != 0).sum()) == m
            bucket.allreduce_end()
            torch.cuda.synchronize()
            assert torch.equal(bucket.flat, before)
    finally:
        dist.destroy_process_group()


def test_sparse_zero_clears_every_written_row(cuda_device, monkeypatch):
    """GradBucket.zero() on a row-major GPU bucket clears only the rows written since its last clear when every
    writer recorded them (gs_grads.dirty_rows from the batched backward's live set; the sparse all-reduce's
    scatter), else all of it: after every step's zero() the whole bucket is 0 — with the live set moving from
    step to step (other cameras), a torch write into a .grad in between (version change: a full clear) and a
    per-view fused backward (an unrecorded writer: a full clear).  The step's gradients equal those of a
    bucket cleared in full every time (DGE_AMD_SPARSE_ZERO=0)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, W, H = 60_000, 160, 120
    g = torch.Generator().manual_seed(2)
    seeds = [torch.randn(3, H, W, generator=g).to(dev) for _ in range(3)]
    bg = torch.zeros(3, device=dev)

    def run(sparse):
        monkeypatch.setattr(mv, "_SPARSE_ZERO", sparse)
        sc = synthetic_scene(P, seed=4, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
        bucket = mv.GradBucket(sc.parameters())
        assert bucket.rows is not None and bucket._dirty is not None
        snaps = []
        for step in range(5):
            bucket.zero()
            torch.cuda.synchronize()
            assert int(torch.count_nonzero(bucket.flat)) == 0, f"step {step}: rows left after zero()"
            cams = [orbit_camera(k + step, 8, W, H, device=dev) for k in range(3)]
            if step == 3:  # a per-view fused backward: writes .grad without recording rows
                (render(cams[0], sc, PipelineParams(), bg)["render"] * seeds[0]).sum().backward()
            else:
                outs = mv.render_views(cams, sc, PipelineParams(), bg, streams=3, speculate=True)
                torch.autograd.backward([o["render"] for o in outs], seeds)
                assert outs.check()
            if step == 1:
                with torch.no_grad():
                    sc._opacity.grad.mul_(1.0)  # (a torch write: the buffer's version moves)
            snaps.append(bucket.flat.clone())
        return snaps

    a, b = run(True), run(False)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert any(bool(x.abs().sum() > 0) for x in a)
