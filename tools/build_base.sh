#!/bin/bash
# Build libgs_raster.so from the sources of a commit (default HEAD) into dge_amd/lib/var/base.so: the
# "base" side of tools/gpu_ab.sh (A/B of the working tree's kernels against a committed build).
set -e
rev=${1:-HEAD}
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp=$(mktemp -d /tmp/gsbase.XXXX)
git -C "$root" archive "$rev" dge_amd/csrc include | tar -x -C "$tmp"
cd "$tmp/dge_amd/csrc"
make -s -j8 LIB=../lib/libgs_raster.so >/dev/null
mkdir -p "$root/dge_amd/lib/var"
cp "$tmp/dge_amd/lib/libgs_raster.so" "$root/dge_amd/lib/var/base.so"
rm -rf "$tmp"
echo "built dge_amd/lib/var/base.so from $rev"
