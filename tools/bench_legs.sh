#!/bin/bash
# Secondary bench legs (not the headline line): BASELINE configs[1], [3] (one GPU's shard), [4],
# the exact-integrator mode and the large-N points. Each leg under its own time limit.
TAG=${1:-legs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ]; then tail -5 "$OUT/$name.err"; exit "$rc"; fi
}
run rollout_fp32 --mode rollout
run rollout_fp16x3 --mode rollout --policy-dtype fp16x3
run rollout_bf16 --mode rollout --policy-dtype bf16
run rollout_2launch --mode rollout --rollout-two-launch
run euler3_4096 --model 3DOF --integrator euler --n 4096
run rk4_3dof_4096 --model 3DOF --n 4096
run n524288 --n 524288
run n4194304 --n 4194304 --steps 500
run dopri5 --integrator dopri5 --steps 200
echo done
