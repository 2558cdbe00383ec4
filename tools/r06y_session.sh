#!/bin/bash
# PPO gradient kernel with the MFMA accumulators in VGPRs (-amdgpu-mfma-vgpr-form, tools/ab/lib_vf.so)
# against the tree: bitwise, phase clocks of both, rollout-bench PPO legs interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06y"; mkdir -p "$OUT"
timeout -k 10 300 python tools/ppo_grad_bitwise.py --libs tree,tools/ab/lib_vf.so --out "$OUT/bitwise.json" > "$OUT/bitwise.log" 2>&1
rc=$?; tail -1 "$OUT/bitwise.log"; [ $rc -gt 1 ] && exit $rc
for v in stamps stamps_vf; do
  RR_LIB_PATH=$R/tools/ab/lib_$v.so timeout -k 10 300 python tools/ppo_stamps.py --out "$OUT/ppo_$v.json" > "$OUT/ppo_$v.log" 2>&1 || exit 3
done
for rep in 1 2; do
  for v in tree vf; do
    lib="$R/rl_rocket_amd/librocket_hip.so"; [ $v = vf ] && lib="$R/tools/ab/lib_vf.so"
    RR_LIB_PATH=$lib timeout -k 10 300 python bench.py --mode rollout --steps 32 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || { tail -20 "$OUT/${v}_$rep.err"; exit 3; }
    python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
u=d['ppo_update']; t=d['train_iteration']
print(sys.argv[2], 'collect', round(d['value']/1e9,3), 'G', 'minibatch us %.2f' % (u['fused_ms_per_minibatch']*1e3), 'train it ms %.3f' % t['ms_per_iteration'])
" "$OUT/${v}_$rep.json" "${v}_$rep" | tee -a "$OUT/summary.txt"
  done
done
echo done
