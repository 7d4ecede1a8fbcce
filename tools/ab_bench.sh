#!/bin/bash
# Same-box A/B of bench.py between the in-tree library and variant builds (tools/build_rev.sh).
# usage: tools/ab_bench.sh "BENCH ARGS" REV [REV ...]     (prints value per library, alternating twice)
set -o pipefail
args=$1; shift
for round in 1 2; do
  for lib in "" "$@"; do
    if [ -n "$lib" ]; then export ORBFE_LIB=pyorbslam_amd/_lib/variants/$lib/liborbfe.so; else unset ORBFE_LIB; fi
    v=$(timeout -k 10 150 python bench.py $args --cpu-sample 0 --allow-dev-env 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'] or round(d['config']['total_pairs_per_step'] / d['dev_env_ms_per_step'] * 1e3, 1))") || exit 1
    echo "round $round lib ${lib:-HEAD-tree} [$args] -> $v"
  done
done
