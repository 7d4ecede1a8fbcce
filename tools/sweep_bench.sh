# bench sweep over handles per GPU / blur side stream (development aid; runs on the GPU box)
set -o pipefail
for cfg in "256 4 1" "256 4 0" "256 8 0" "256 2 0" "256 4 0 --no-prof" "512 8 0" "512 4 0"; do
  set -- $cfg
  r=$(timeout -k 10 120 python bench.py --pairs $1 --streams $2 --blur-fork $3 $4 --cpu-sample 0 --steps 15 --warmup 4 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "pairs=$1 streams=$2 blur_fork=$3 $4 -> $r"
done
