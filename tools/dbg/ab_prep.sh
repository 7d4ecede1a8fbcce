#!/bin/bash
# Build liborbfe.so of git revision REV into _ab/NAME/ (a top-level scratch directory that travels with gpurun,
# unlike pyorbslam_amd/_lib/variants/; git-ignored; delete it after the A/B).  usage: tools/dbg/ab_prep.sh REV NAME
set -e
rev=$1; name=${2:-$1}
root=$(cd "$(dirname "$0")/../.." && pwd)
out=$root/_ab/$name
tmp=$(mktemp -d)
git -C "$root" archive "$rev" pyorbslam_amd/csrc include Makefile | tar -x -C "$tmp"
make -s -C "$tmp" pyorbslam_amd/_lib/liborbfe.so -j8
mkdir -p "$out"
cp "$tmp/pyorbslam_amd/_lib/liborbfe.so" "$out/"
rm -rf "$tmp"
echo "$out/liborbfe.so"
