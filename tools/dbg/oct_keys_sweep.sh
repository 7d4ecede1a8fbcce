# Debug aid: default bench (4 handles) with the octree's LDS candidate capacity overridden (ORBFE_OCT_KEYS),
# interleaved rounds; prints pairs/s and the standalone octree ms.
set -o pipefail
for r in 1 2 3; do
  for k in ${OCT_KEYS:-7424 0 2048 4096}; do
    v=$(ORBFE_OCT_KEYS=$k timeout -k 10 150 python bench.py --cpu-sample 0 --no-parity 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_standalone_step']['octree'])") || exit 1
    echo "round $r oct_keys=$k -> $v"
  done
done
