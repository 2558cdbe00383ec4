#!/bin/bash
# kernel timeline of the fused graphed PPO epoch (rollout bench with PPO): per-minibatch kernels and gaps
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06j"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp" -o rp -- python "$R/bench.py" --mode rollout --steps 32 > "$OUT/rollout.json" 2> "$OUT/rollout.err" || exit $?
