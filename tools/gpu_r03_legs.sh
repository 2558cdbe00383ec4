#!/bin/bash
# Round-3 secondary legs on one GPU (each step time-bounded; a failure ends the script).
TAG=${1:-r03legs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "$name failed ($?)"; exit 1; }
  python -c "
import json; d=[json.loads(l) for l in open('$O/$name.json') if l.startswith('{')][-1]; r=d.get('roofline') or {}
print('%-22s %8.3f G %9.3f us/step  frac %.4f  frac_wall %.4f' % ('$name', d['value']/1e9, d['ms_per_step']*1e3, r.get('frac') or 0, r.get('frac_wall') or 0))" | tee -a "$O/summary.txt"
}
run headline_k20_a --steps 20 --warmup 5
run headline_k20_b --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs
run headline_k2000 --no-cpu-baseline --no-sb3-legs
run n524288 --n 524288 --steps 500 --warmup 20 --no-cpu-baseline --no-sb3-legs
run dof3_n524288 --model 3DOF --n 524288 --steps 500 --warmup 20 --no-cpu-baseline
run cfg1_3dof_euler --model 3DOF --integrator euler --n 4096 --no-cpu-baseline
run cfg1_3dof_rk4 --model 3DOF --n 4096 --no-cpu-baseline
run exact_dopri5 --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline
run rollout_fp32 --mode rollout --steps 320
run rollout_fp16x3 --mode rollout --steps 320 --policy-dtype fp16x3
run rollout_bf16 --mode rollout --steps 320 --policy-dtype bf16
run gather_w1 --gather-leg --steps 2000 --no-cpu-baseline --no-sb3-legs
export RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo
run gpus2_gloo --gpus 2 --steps 20 --warmup 5
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29617 tools/dist_check.py > "$O/dist_check_gloo2.json" 2> "$O/dist_check_gloo2.err" || { echo "dist_check failed"; exit 1; }
cat "$O/dist_check_gloo2.json" | tee -a "$O/summary.txt"
echo done
