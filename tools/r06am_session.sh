#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06am"; mkdir -p "$OUT"
python -c "import torch; print('prio range', torch.cuda.Stream.priority_range())"
for rep in 1 2; do
  for v in 0 1; do
    RR_PERM_HI=$v timeout -k 10 300 python bench.py --mode rollout --steps 32 > "$OUT/hi${v}_$rep.json" 2> "$OUT/hi${v}_$rep.err" || { tail -20 "$OUT/hi${v}_$rep.err"; exit 3; }
    python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
u=d['ppo_update']; t=d['train_iteration']
print(sys.argv[2], 'minibatch us %.2f' % (u['fused_ms_per_minibatch']*1e3), 'train it ms %.3f' % t['ms_per_iteration'])
" "$OUT/hi${v}_$rep.json" "hi${v}_$rep" | tee -a "$OUT/summary.txt"
  done
done
