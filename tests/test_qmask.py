"""The emission's quadrant mask (dge_amd/csrc/gs_qmask.h) never drops a quadrant the blend uses.

tests/qmask_check.cpp brute-forces the blend's per-pixel skip tests (forward.cu:336-348, with the
oracle's exp) over the 64 pixels of every quadrant for random Gaussians around a tile — elongated,
tiny and huge footprints, opacities at the 1/255 threshold, tile origins at 2k-pixel coordinates —
and counts quadrants some pixel blends whose mask bit is clear.  Also reported: how many more
quadrants the mask keeps than the blend's former per-wave cull (cull_keep), which is the cost side.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def qmask_bin(tmp_path_factory):
    lib = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s"], check=True)
    out = str(tmp_path_factory.mktemp("qmask") / "qmask_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", out, os.path.join(ROOT, "tests", "qmask_check.cpp"),
                    "-L" + os.path.dirname(lib), "-loracle", "-Wl,-rpath," + os.path.dirname(lib), "-lm"], check=True)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_quadrant_mask_is_conservative(qmask_bin, seed):
    r = subprocess.run([qmask_bin, "400000", str(seed)], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    last = r.stdout.strip().splitlines()[-1]
    f = dict(zip(last.split()[0::2], last.split()[1::2]))
    assert int(f["misses"]) == 0
    assert int(f["quadrants_needed"]) > 100000  # (the cases do exercise the bound)
