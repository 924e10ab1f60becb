"""Build check (CPU): no kernel of the built library uses scratch (private segment) memory.

A spill to scratch in a hot kernel costs it several us per launch at c2 and has crept in twice after
unrelated edits (the blend's register budget is at its 3-waves-per-SIMD limit), so the shipped
library is inspected directly: the `.hip_fatbin` section of libgs_raster.so holds one offload bundle
per translation unit; each bundle's gfx950 code object lists every kernel's
`.private_segment_fixed_size` in its metadata notes.
"""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "dge_amd", "lib", "libgs_raster.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.access(p, os.X_OK) else None


def kernel_scratch(lib: str) -> dict:
    """{kernel symbol: private segment bytes} over every gfx950 code object in `lib`."""
    objcopy, bundler, readelf = _tool("llvm-objcopy"), _tool("clang-offload-bundler"), _tool("llvm-readelf")
    if not (objcopy and bundler and readelf):
        pytest.skip("LLVM tools not found under /opt/rocm/lib/llvm/bin")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(d, "stripped")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        assert starts, "no offload bundle in .hip_fatbin"
        for i, s in enumerate(starts):
            piece = os.path.join(d, f"b{i}.bin")
            with open(piece, "wb") as f:
                f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"b{i}.hsaco")
            r = subprocess.run([bundler, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                                f"--input={piece}", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            notes = subprocess.run([readelf, "--notes", co], check=True, capture_output=True, text=True).stdout
            # each kernel's metadata map lists .name and .private_segment_fixed_size (in either order)
            for block in notes.split("  - .")[1:]:
                name = re.search(r"\.name:\s+(\S+)", "." + block)
                priv = re.search(r"\.private_segment_fixed_size:\s+(\d+)", "." + block)
                if name and priv:
                    out[name.group(1)] = int(priv.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(LIB), reason="libgs_raster.so not built")
def test_no_kernel_uses_scratch():
    sizes = kernel_scratch(LIB)
    assert any("k_render_fwd" in k for k in sizes) and any("k_render_bwd" in k for k in sizes), sorted(sizes)[:10]
    spilled = {k: v for k, v in sizes.items() if v}
    assert not spilled, f"kernels with scratch: {spilled}"
