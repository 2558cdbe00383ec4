#!/bin/bash
# The next epoch's permutation drawn on a side stream during the replay: learner / rollout tests,
# then the rollout bench's PPO legs twice
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06an"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_rollout.py -x -v --timeout 300 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -30; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --mode rollout --steps 32 > "$OUT/tree_$rep.json" 2> "$OUT/tree_$rep.err" || { tail -20 "$OUT/tree_$rep.err"; exit 3; }
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
u=d['ppo_update']; t=d['train_iteration']
print(sys.argv[2], 'minibatch us %.2f' % (u['fused_ms_per_minibatch']*1e3), 'train it ms %.3f' % t['ms_per_iteration'], '%.4g env-steps/s' % t['value'])
" "$OUT/tree_$rep.json" "tree_$rep" | tee -a "$OUT/summary.txt"
done
echo done
