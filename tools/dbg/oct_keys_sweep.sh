set -o pipefail
for k in 7424 0 2048 7424 0; do
  v=$(ORBFE_OCT_KEYS=$k timeout -k 10 150 python bench.py --cpu-sample 0 --no-parity 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms_standalone_step']['octree'])") || exit 1
  echo "oct_keys=$k -> $v"
done
