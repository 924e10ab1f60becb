"""Which side of the speculated, batched-backward mismatch is wrong (dev probe, GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd import gaussian_renderer as GR  # noqa: E402
from dge_amd.diff_gaussian_rasterization import set_fused_grad_accumulation  # noqa: E402
from fused_accum_debug import names, run  # noqa: E402

GR._SPEC_RENDER = False
ref = run(True, False, True)
ref_sep = run(True, False, False)
GR._SPEC_RENDER = True
a = run(True, False, True)
b = run(False, False, True)
for tag, got in (("spec fused", a), ("spec autograd", b)):
    print(tag, "vs exact:", [(n, int((x != y).sum())) for n, x, y in zip(names, got, ref) if not torch.equal(x, y)])
# per-view gradients alone (separate backward, spec) summed in both orders
print("exact joint vs separate:", [(n, int((x != y).sum())) for n, x, y in zip(names, ref, ref_sep) if not torch.equal(x, y)])
