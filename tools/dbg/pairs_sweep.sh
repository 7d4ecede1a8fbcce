# Debug aid: default bench at several batch sizes (pairs per step), interleaved rounds.
set -o pipefail
for r in 1 2; do
  for p in ${PAIRS:-256 512 1024}; do
    v=$(timeout -k 10 200 python bench.py --cpu-sample 0 --no-parity --roofline-steps 0 --pairs $p 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "round $r pairs=$p -> $v"
  done
done
