set -o pipefail
for r in 1 2; do
for s in 2 3 4 6 8; do
  v=$(timeout -k 10 120 python bench.py --streams $s --cpu-sample 0 --no-c3 --no-c4 --no-c5 --no-host-fed --no-parity --roofline-steps 0 --steps 40 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "round $r streams $s: $v"
done; done
