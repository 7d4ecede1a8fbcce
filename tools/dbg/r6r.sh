# handles (streams) x lanes sweep of the headline step on the final build, 2 alternating rounds
mkdir -p gpurun_out/r6r
for r in 1 2; do for cfg in "4 1" "3 1" "5 1" "6 1" "8 1" "4 2" "2 2"; do
  set -- $cfg
  v=$(timeout -k 10 150 python bench.py --streams $1 --lanes $2 --steps 30 --warmup 5 --no-parity --roofline-steps 0 --no-c4 --no-host-fed --no-c3 --no-c5 --cpu-sample 0 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
  echo "round $r streams $1 lanes $2: $v" >> gpurun_out/r6r/sweep.log
done; done
cat gpurun_out/r6r/sweep.log
