set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for cfg in "512 4" "640 5" "768 6" "512 2" "768 3"; do
  set -- $cfg
  v=$(timeout -k 10 150 python bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-parity --roofline-steps 0 --pairs $1 --streams $2 2>/dev/null | tail -1 | python -c "import sys,json; print(json.loads(sys.stdin.read())['value'])") || exit 1
  echo "round $r pairs $1 handles $2 -> $v"
done
done
