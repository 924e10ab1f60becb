"""GPU tests of the sparse-row gradient exchange kernels (gs_rows_live / gs_rows_gather /
gs_rows_scatter, dge_amd/csrc/gs_bucket.hip) against the torch formulation GradBucket uses on CPU:
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
