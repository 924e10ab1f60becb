"""cProfile of DGE's own loop shape on the fused render() (dev probe, GPU): bench.py's dge_loop_unchanged leg
(threestudio/systems/DGE.py forward() :170-239 per view: training render, radii max, semantic render with
the edit mask as override_color, its norm > 0.8 map, the boolean-mask visualisation; then the masked l1
and one backward).  Prints the loop's wall time per view and the host functions by own time."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
P, W, H, V = 1_000_000, 512, 512, 3
sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
bg = torch.zeros(3, device=dev)
pipe = PipelineParams()
sc.mask = (torch.rand(P, generator=torch.Generator().manual_seed(5)) < 0.2).to(dev)
gts = [torch.rand(H, W, 3, generator=torch.Generator().manual_seed(50 + i)).to(dev) for i in range(V)]


def loop():
    for p in sc.parameters():
        p.grad = None
    images, masks, radii = [], [], None
    for i, cam in enumerate(cams):
        pkg = render(cam, sc, pipe, bg)
        image, r = pkg["render"], pkg["radii"]
        radii = r if i == 0 else torch.max(r, radii)
        sm = render(cam, sc, pipe, bg, override_color=sc.mask[..., None].float().repeat(1, 3))["render"]
        sm = torch.norm(sm, dim=0) > 0.8
        viz = image.detach().clone().permute(1, 2, 0)
        viz[sm] = 0.40 * viz[sm] + 0.60 * torch.tensor([1.0, 0.0, 0.0], device=dev)
        masks.append(sm)
        images.append(image.permute(1, 2, 0))
    images = torch.stack(images, 0)
    m = torch.stack(masks, 0)[..., None].float()
    loss = torch.nn.functional.l1_loss(images * m, torch.stack(gts, 0) * m)
    loss.backward()


for _ in range(5):
    loop()
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    loop()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"dge loop: {n * V / dt:.1f} views/s, {dt / (n * V) * 1e6:.0f} us per view")
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    loop()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(35)
