#!/bin/bash
# PPO learner: the chained whole-minibatch call (rr_ppo_update) — its tests, the A/B against
# rr_ppo_grad + rr_clip_adam, the rollout bench's PPO legs and a rocprofv3 trace of the update
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06s"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_rollout.py -x -v --timeout 300 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -30; exit $rc; }
timeout -k 10 300 python tools/ppo_chain_ab.py --out "$OUT/ppo_chain_ab.json" > "$OUT/ppo_chain_ab.log" 2>&1 || { tail -20 "$OUT/ppo_chain_ab.log"; exit 3; }
tail -1 "$OUT/ppo_chain_ab.log"
timeout -k 10 300 python bench.py --mode rollout --steps 32 > "$OUT/rollout.json" 2> "$OUT/rollout.err" || { tail -20 "$OUT/rollout.err"; exit 3; }
python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
u=d['ppo_update']; t=d['train_iteration']
print('minibatch us %.2f' % (u['fused_ms_per_minibatch']*1e3), 'epoch ms %.3f' % u['fused_graphed_epoch_ms'], 'train it ms %.3f' % t['ms_per_iteration'], '%.3e env-steps/s' % t['value'])
" "$OUT/rollout.json" | tee "$OUT/summary.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o ppo -- python3 "$R/tools/ppo_chain_ab.py" --reps 1 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 3; }
echo done
