#!/bin/bash
# Step throughput over (pairs per step, handles) on one box, alternating rounds (pairs/s per config).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for r in 1 2; do
  for cfg in "512 4" "512 3" "512 6" "512 8" "768 6" "1024 4" "1024 8"; do
    set -- $cfg
    v=$(timeout -k 10 120 python bench.py --pairs $1 --streams $2 --steps 20 --warmup 3 --cpu-sample 0 --no-parity --roofline-steps 0 --no-c4 --no-host-fed --no-c3 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "round $r pairs $1 streams $2: $v"
  done
done
