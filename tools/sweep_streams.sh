set -o pipefail
for s in 1 2 4 8; do
  v=$(timeout -k 10 150 python bench.py --streams $s --cpu-sample 0 --no-parity --roofline-steps 0 2>/dev/null | tail -1 | python -c "import sys,json; print(json.loads(sys.stdin.read())['value'])") || exit 1
  echo "streams $s -> $v"
done
for p in 512; do
  v=$(timeout -k 10 150 python bench.py --pairs $p --cpu-sample 0 --no-parity --roofline-steps 0 2>/dev/null | tail -1 | python -c "import sys,json; print(json.loads(sys.stdin.read())['value'])") || exit 1
  echo "pairs $p streams 4 -> $v"
done
