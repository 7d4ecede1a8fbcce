#!/bin/bash
# Same-box kernel-trace A/B of the small-batch chain (tools/small_trace.py, rocprofv3 --kernel-trace) between the
# in-tree library and variants: per-kernel median durations (tools/ktrace_steps.py) for each.
# usage: bash tools/dbg/trace_ab.sh OUT "SMALL_TRACE_ARGS" NAME [NAME ...]   (NAME "tree" = the in-tree library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=$1; args=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$out"
for lib in "$@"; do
  if [ "$lib" = tree ]; then unset ORBFE_LIB; else export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/$lib" -o run -- python tools/small_trace.py $args \
    > "$out/$lib.log" 2>&1 || exit 1
  echo "== $lib ($args)"
  python tools/ktrace_steps.py "$out/$lib" 5 | tail -8
done
