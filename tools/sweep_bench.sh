# bench sweep over pairs per step / handles per GPU (development aid; runs on the GPU box)
set -o pipefail
for cfg in "256 4" "512 4" "512 8" "768 4" "1024 4" "1024 8"; do
  set -- $cfg
  r=$(timeout -k 10 120 python bench.py --pairs $1 --streams $2 --cpu-sample 0 --steps 15 --warmup 4 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "pairs=$1 streams=$2 -> $r"
done
