#!/bin/bash
# PMC passes for one command (development aid). usage: tools/pmc_run.sh OUTDIR "COUNTERS ..." [more counter sets ...] -- cmd...
# Each counter set is its own rocprofv3 --pmc run (never combined with sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; shift
sets=()
while [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
export TMPDIR=/tmp
mkdir -p "$out"
i=0
for s in "${sets[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $s --output-format csv -d "$out/p$i" -o run -- "$@" > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($s) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
  i=$((i+1))
done
