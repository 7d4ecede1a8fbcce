#!/bin/bash
# GPU session script for gpurun: parity tests, then a short bench, then (optionally) a rocprof summary.
# Stops at the first step that faults, aborts or times out (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
stage() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name (timeout ${to}s) $(date +%T)"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! stopping after $name (rc=$rc)"; exit $rc; fi
  return $rc
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  stage pytest_gpu 900 python -m pytest tests -m gpu -q -rf || { [ "$MODE" = test ] && exit 1; }
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  stage bench 600 python bench.py --steps 10 --warmup 3 --cpu-sample 2
fi
if [ "$MODE" = dist2 ]; then
  # rehearse the N>1 path on one GPU: 2 ranks over gloo on cuda:0 (never the N=8 case)
  ORBFE_DIST_BACKEND=gloo stage dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --pairs 16 --gather
fi
if [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  stage rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 --cpu-sample 0
fi
exit 0
