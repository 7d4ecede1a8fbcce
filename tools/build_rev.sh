#!/bin/bash
# Build liborbfe.so of git revision REV into pyorbslam_amd/_lib/variants/REV/ (for ORBFE_LIB A/B runs).
# usage: tools/build_rev.sh REV
set -e
rev=$1
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/pyorbslam_amd/_lib/variants/$rev
tmp=$(mktemp -d)
git -C "$root" archive "$rev" pyorbslam_amd/csrc include Makefile | tar -x -C "$tmp"
make -s -C "$tmp" pyorbslam_amd/_lib/liborbfe.so -j8
mkdir -p "$out"
cp "$tmp/pyorbslam_amd/_lib/liborbfe.so" "$out/"
rm -rf "$tmp"
echo "$out/liborbfe.so"
