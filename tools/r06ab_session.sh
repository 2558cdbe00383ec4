#!/bin/bash
# The learner's kernels in the collect TU (MFMA accumulators in VGPRs): learner / rollout tests,
# bitwise vs the previous build, phase clocks, rollout-bench PPO legs of both builds interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06ai"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_rollout.py -x -v --timeout 300 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -1 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -30; exit $rc; }
timeout -k 10 300 python tools/ppo_grad_bitwise.py --libs tree,tools/ab/lib_prev.so --out "$OUT/bitwise.json" > "$OUT/bitwise.log" 2>&1
rc=$?; tail -1 "$OUT/bitwise.log"; [ $rc -gt 1 ] && exit $rc
RR_LIB_PATH=$R/tools/ab/lib_stamps.so timeout -k 10 300 python tools/ppo_stamps.py --out "$OUT/ppo_stamps.json" > "$OUT/ppo_stamps.log" 2>&1 || exit 3
for rep in 1 2; do
  for v in tree prev; do
    lib="$R/rl_rocket_amd/librocket_hip.so"; [ $v = prev ] && lib="$R/tools/ab/lib_prev.so"
    RR_LIB_PATH=$lib timeout -k 10 300 python bench.py --mode rollout --steps 32 > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || { tail -20 "$OUT/${v}_$rep.err"; exit 3; }
    python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
u=d['ppo_update']; t=d['train_iteration']
print(sys.argv[2], 'minibatch us %.2f' % (u['fused_ms_per_minibatch']*1e3), 'train it ms %.3f' % t['ms_per_iteration'], '%.4g env-steps/s' % t['value'])
" "$OUT/${v}_$rep.json" "${v}_$rep" | tee -a "$OUT/summary.txt"
  done
done
echo done
