#!/bin/bash
# Build an A/B variant of libgs_raster.so with extra preprocessor flags:
#   tools/build_variant.sh NAME "-DFLAG ..."  ->  dge_amd/lib/var/NAME.so
set -e
cd "$(dirname "$0")/../dge_amd/csrc"
make -s -j8
name=$1; shift
mkdir -p build/var/$name ../lib/var
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-function -fno-gpu-rdc -munsafe-fp-atomics"
objs=""
for src in gs_api gs_preprocess gs_sort gs_render gs_backward gs_optim gs_bucket; do
  /opt/rocm/bin/hipcc $HIPFLAGS "$@" -c $src.hip -o build/var/$name/$src.o &
  objs="$objs build/var/$name/$src.o"
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../lib/var/$name.so $objs
echo "built dge_amd/lib/var/$name.so"
