#!/bin/bash
# GPU evidence for one revision of the default bench: parity tests, the bench line, a rocprofv3 kernel
# trace of the same command, and the FETCH_SIZE / WRITE_SIZE passes (one pass each, as
# MI355X_MICROARCH.md prescribes) that profiles/traffic.json is built from.
# usage (on the GPU box): bash tools/evidence.sh TAG      -> gpurun_out/ev_TAG/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-run}
out=gpurun_out/ev_$tag
mkdir -p "$out"
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 5"
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 300 python $BENCH --cpu-sample 64
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run -- python $BENCH --cpu-sample 0
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- python bench.py --steps 4 --warmup 1 --cpu-sample 0
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- python bench.py --steps 4 --warmup 1 --cpu-sample 0
echo "evidence done"
