#!/bin/bash
# PPO minibatch optimizer half: one-launch clip + Adam (adam_fused_kernel, in-tree) against the two-launch
# path (RR_ADAM_TWO_LAUNCH=1): the PPO tests, then the rollout bench's fused PPO legs, interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06l"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -x -q --timeout 300 --timeout-method thread -m gpu > "$OUT/test_ppo.log" 2>&1 || { tail -30 "$OUT/test_ppo.log"; exit 1; }
tail -1 "$OUT/test_ppo.log"
for rep in 1 2; do
  for v in fused two; do
    if [ $v = two ]; then export RR_ADAM_TWO_LAUNCH=1; else unset RR_ADAM_TWO_LAUNCH; fi
    timeout -k 10 300 python bench.py --mode rollout --steps 32 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || exit $?
    python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
u=d['ppo_update']; t=d['train_iteration']
print(sys.argv[2], 'minibatch us %.2f' % (u['fused_ms_per_minibatch']*1e3), 'epoch ms %.3f' % u['fused_graphed_epoch_ms'], 'train it ms %.3f' % t['ms_per_iteration'], '%.3e env-steps/s' % t['value'])
" "$OUT/${v}_$rep.json" "${v}_$rep" | tee -a "$OUT/summary.txt"
  done
done
