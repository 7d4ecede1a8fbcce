#!/bin/bash
# GPU evidence for one revision: parity tests, the default bench line (throughput + its own parity sample +
# C4 / C4 rank share / C5 EuRoC / host-fed / C3 / standalone per-stage roofline / cpu_baseline), the C3
# frame-mode line, the launcher refusal and a 2-rank gloo run, rocprofv3 kernel traces (default bench, the
# 8-pair share, the frame path, the C3 replay's frames), and the PMC passes (one counter group per pass, MI355X_MICROARCH.md) over the
# standalone pass (--roofline-only) for KITTI and EuRoC: FETCH_SIZE, WRITE_SIZE (profiles/traffic.json via
# tools/traffic.py), SQ_INSTS_VALU + SQ_INSTS_LDS + GRBM_GUI_ACTIVE, and the busy-cycle group
# SQ_ACTIVE_INST_VALU + SQ_BUSY_CYCLES + SQ_WAIT_INST_ANY + GRBM_GUI_ACTIVE (profiles/valu.json via tools/valu.py).
# usage (on the GPU box): bash tools/evidence.sh TAG [PART]   -> gpurun_out/ev_TAG/
#   PART: all (default), a (tests, bench lines, launcher runs, kernel traces), b (PMC passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-run}
part=${2:-all}
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
if [ "$part" != b ]; then
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 500 python bench.py
step bench_frame 300 python bench.py --mode frame --steps 96 --warmup 1
# `--gpus 2` on this one-GPU box must refuse (exit 2), never report one rank as two
echo "== bench_gpus2_refuses $(date +%T)"
timeout -k 10 120 python bench.py --gpus 2 > "$out/bench_gpus2_refuses.log" 2>&1; rc=$?
echo "== bench_gpus2_refuses rc=$rc (expected 2)"; tail -n 2 "$out/bench_gpus2_refuses.log"
[ $rc -eq 2 ] || exit 1
step bench_gpus2_gloo 300 env ORBFE_DIST_BACKEND=gloo python bench.py --gpus 2 --pairs 64 --steps 5 --warmup 2 --no-parity --roofline-steps 0
step bench_c4_gloo8 300 env ORBFE_DIST_BACKEND=gloo OMP_NUM_THREADS=2 python bench.py --gpus 8 --total-pairs 64 --pairs 8 --steps 3 --warmup 1 --cpu-sample 0 --no-c3 --no-host-fed --roofline-steps 1
step rccl_single 150 python tools/rccl_probe.py --single
step ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ktrace" -o run -- python bench.py --cpu-sample 0 --no-c4 --no-host-fed --no-c3 --no-c5
step ktrace_share8 120 rocprofv3 --kernel-trace --output-format csv -d "$out/ktrace_share8" -o run -- python tools/small_trace.py --pairs 8 --steps 50
step ktrace_frame 120 rocprofv3 --kernel-trace --output-format csv -d "$out/ktrace_frame" -o run -- python tools/small_trace.py --frame --steps 50
step ktrace_c3 200 rocprofv3 --kernel-trace --output-format csv -d "$out/ktrace_c3" -o run -- python bench.py --mode frame --steps 96 --warmup 1
step ktrace_share8x2 120 rocprofv3 --kernel-trace --output-format csv -d "$out/ktrace_share8x2" -o run -- python tools/small_trace.py --pairs 8 --steps 50 --graphs 0 --handles 2
step host_fed_trace 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$out/host_fed_trace" -o run -- python tools/host_fed_trace.py --steps 8
fi
[ "$part" = a ] && { echo "evidence done (part a)"; exit 0; }
for cam in kitti euroc; do
  args="--roofline-only --roofline-steps 2"
  [ $cam = euroc ] && args="$args --width 752 --height 480 --nfeatures 1000"
  step pmc_${cam}_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_$cam/fetch" -o run -- python bench.py $args
  step pmc_${cam}_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_$cam/write" -o run -- python bench.py $args
  step pmc_${cam}_valu 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_$cam/valu" -o run -- python bench.py $args
  step pmc_${cam}_busy 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc_$cam/busy" -o run -- python bench.py $args
done
echo "evidence done"
