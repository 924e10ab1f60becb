"""dge_amd — MI355X-native differentiable 3D Gaussian Splatting rasterizer.

The hot path of bonapark00/DGE (gaussian_renderer.render() -> the vendored
diff-gaussian-rasterization extension) rebuilt as hand-written HIP kernels
for gfx950 behind a C ABI (include/gs_raster.h), with the reference's Python
surface on top:

  dge_amd.diff_gaussian_rasterization  drop-in for the reference package
  dge_amd.gaussian_renderer            render(), camera2rasterizer(), point_cloud_render()
  dge_amd.cameras / scene / sh_utils   the caller-side inputs of the path
  dge_amd.multiview                    view-sharded multi-GPU step (RCCL all-reduce)
"""
from . import _native  # noqa: F401

__version__ = "0.1.0"


def install_alias() -> None:
    """Make ``import diff_gaussian_rasterization`` resolve to this package.

    DGE's renderer (gaussiansplatting/gaussian_renderer/__init__.py:14-17)
    imports the rasterizer under that name; after this call it gets the
    gfx950 implementation with no change to DGE's code.
    """
    import sys

    from . import _C, diff_gaussian_rasterization

    sys.modules["diff_gaussian_rasterization"] = diff_gaussian_rasterization
    sys.modules["diff_gaussian_rasterization._C"] = _C
