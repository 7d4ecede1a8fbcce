#!/bin/bash
# Build the WORKING TREE's liborbfe.so with extra compiler defines into pyorbslam_amd/_lib/variants/NAME/
# (experiment switches compiled out of the production build; every variant build defines ORBFE_DEV_VARIANTS,
# which adds the microbench ablation kernels; A/B with tools/dbg/lib_ab.sh NAME).
# usage: tools/dbg/build_variant.sh NAME "-DFOO -DBAR=2"
set -e
name=$1
defs=$2
root=$(cd "$(dirname "$0")/../.." && pwd)
out=$root/pyorbslam_amd/_lib/variants/$name
# AB=1: into _ab/NAME instead (travels with gpurun; tools/dbg/ab.sh)
[ "${AB:-0}" = 1 ] && out=$root/_ab/$name
tmp=$(mktemp -d)
cp -r "$root/pyorbslam_amd" "$root/include" "$root/Makefile" "$tmp/"
rm -rf "$tmp/pyorbslam_amd/_lib"
mkdir -p "$tmp/pyorbslam_amd/_lib"
make -s -C "$tmp" pyorbslam_amd/_lib/liborbfe.so -j8 \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -munsafe-fp-atomics -Wno-unused-result -DORBFE_DEV_VARIANTS $defs" 2>&1 |
  grep -v "warning\|note:\|^ *|\|^ *[0-9]* |\|generated" || true
mkdir -p "$out"
cp "$tmp/pyorbslam_amd/_lib/liborbfe.so" "$out/"
rm -rf "$tmp"
echo "$out/liborbfe.so"
