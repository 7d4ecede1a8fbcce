#!/bin/bash
# GPU evidence for one revision: parity tests, the default bench line (throughput + parity check of its own
# workload + standalone per-stage roofline pass + cpu_baseline), the C3 frame-mode line, a gloo 2-rank
# rehearsal with the timed device-side gather, a rocprofv3 kernel trace of the default bench command, and
# FETCH_SIZE / WRITE_SIZE passes (one counter pass each, as MI355X_MICROARCH.md prescribes) over the
# standalone pass only (--roofline-only) that profiles/traffic.json is built from, and an SQ_INSTS_VALU pass
# for profiles/valu.json (tools/valu.py).
# usage (on the GPU box): bash tools/evidence.sh TAG      -> gpurun_out/ev_TAG/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-run}
out=gpurun_out/ev_$tag
mkdir -p "$out"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 to=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "$out/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 400 python bench.py
step bench_euroc 300 python bench.py --width 752 --height 480 --nfeatures 1000 --cpu-sample 12 --no-c3
step bench_frame 300 python bench.py --mode frame --steps 64 --warmup 1
step bench_c4_1gpu 300 python bench.py --total-pairs 64 --cpu-sample 0 --no-c3
# `--gpus 2` on this one-GPU box must refuse (exit 2), never report one rank as two
echo "== bench_gpus2_refuses $(date +%T)"
timeout -k 10 120 python bench.py --gpus 2 > "$out/bench_gpus2_refuses.log" 2>&1; rc=$?
echo "== bench_gpus2_refuses rc=$rc (expected 2)"; tail -n 2 "$out/bench_gpus2_refuses.log"
[ $rc -eq 2 ] || exit 1
# the launcher path with two gloo ranks sharing the GPU: default extras (gather, C4 + gather, host-fed)
step bench_gpus2_gloo 300 env ORBFE_DIST_BACKEND=gloo python bench.py --gpus 2 --pairs 64 --steps 5 --warmup 2 --no-parity --roofline-steps 0
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run -- python bench.py --cpu-sample 0 --no-c4 --no-host-fed --no-c3
step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o run -- python bench.py --roofline-only --roofline-steps 2
step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o run -- python bench.py --roofline-only --roofline-steps 2
step pmc_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_valu" -o run -- python bench.py --roofline-only --roofline-steps 2
step pmc_lds 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --output-format csv -d "$out/pmc_lds" -o run -- python bench.py --roofline-only --roofline-steps 2
EU="--width 752 --height 480 --nfeatures 1000"
step pmc_fetch_euroc 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch_euroc" -o run -- python bench.py --roofline-only --roofline-steps 2 $EU
step pmc_write_euroc 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write_euroc" -o run -- python bench.py --roofline-only --roofline-steps 2 $EU
step pmc_valu_euroc 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_valu_euroc" -o run -- python bench.py --roofline-only --roofline-steps 2 $EU
echo "evidence done"
