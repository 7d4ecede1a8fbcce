#!/bin/bash
# Same-box A/B of the Python host layer: the C3 frame-mode bench with the tree's pyorbslam_amd/*.py against
# those of git revision REV (packed here by `tools/dbg/py_ab.sh --pack REV` into tools/dbg/py_ab_old.tar,
# which travels with the snapshot), same liborbfe.so, alternating.  usage (GPU box): bash tools/dbg/py_ab.sh
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
if [ "$1" = --pack ]; then
  git -C "$root" archive "$2" pyorbslam_amd/*.py > "$root/tools/dbg/py_ab_old.tar"; exit $?
fi
old=/tmp/py_ab_old
rm -rf "$old" && mkdir -p "$old" && cp -r "$root/bench.py" "$root/pyorbslam_amd" "$root/tests" "$root/oracle" "$root/profiles" "$old/" &&
  tar -x -C "$old" -f "$root/tools/dbg/py_ab_old.tar" || exit 1
for r in 1 2 3; do
  for side in tree old; do
    d=$root; [ $side = old ] && d=$old
    v=$(cd "$d" && timeout -k 10 200 python bench.py --mode frame --steps 96 --warmup 1 2>/dev/null | tail -1 |
        python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['latency_ms'])") || exit 1
    echo "round $r $side: $v"
  done
done
