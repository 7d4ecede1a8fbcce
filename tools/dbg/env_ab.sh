#!/bin/bash
# Same-box A/B of a process-level knob (read once per process): VAR=a vs VAR=b on the default 4-handle step
# (tools/dbg/env_sweep.py) and the standalone stage times, alternating.  usage: bash tools/dbg/env_ab.sh VAR a b
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
var=$1; shift
for r in 1 2 3; do
  for v in "$@"; do
    st=$(env "$var=$v" timeout -k 10 120 python tools/dbg/env_sweep.py --var ORBFE_NONE --rounds 2 =0 2>/dev/null | tail -1) || exit 1
    sa=$(env "$var=$v" timeout -k 10 120 python bench.py --roofline-only --cpu-sample 0 2>/dev/null | tail -1 | python -c "import sys,json; print(json.loads(sys.stdin.read())['stage_ms_standalone_step'])") || exit 1
    echo "round $r $var=$v: $st | standalone $sa"
  done
done
