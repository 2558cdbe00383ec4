#!/bin/bash
# Final-tree GPU session: the whole GPU suite, smoke, the driver's default bench command twice,
# a 2000-step bench and the rollout bench (training iteration); the kernels' source hash.
TAG=${1:-r06final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
python -c "from rl_rocket_amd.build import source_hash; print(source_hash())" > "$OUT/source_hash.txt"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "[pytest_gpu] exit $rc" | tee -a "$OUT/status.txt"; tail -1 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" "$OUT/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "[smoke] exit $rc" | tee -a "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_k20_$k.json" 2> "$OUT/bench_k20_$k.err"
  rc=$?; echo "[bench_k20_$k] exit $rc" | tee -a "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python bench.py --steps 2000 --warmup 100 > "$OUT/bench_k2000.json" 2> "$OUT/bench_k2000.err"
rc=$?; echo "[bench_k2000] exit $rc" | tee -a "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --mode rollout --steps 32 > "$OUT/rollout.json" 2> "$OUT/rollout.err"
rc=$?; echo "[rollout] exit $rc" | tee -a "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
python - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
for f in ("bench_k20_1", "bench_k20_2", "bench_k2000"):
    d = [json.loads(l) for l in open("%s/%s.json" % (out, f)) if l.startswith("{")][-1]
    print(f, "value %.4g" % d["value"], "ms/step %.5f" % d["ms_per_step"], "frac %.3f" % d["roofline"]["frac"])
d = [json.loads(l) for l in open(out + "/rollout.json") if l.startswith("{")][-1]
print("rollout value %.4g" % d["value"], "minibatch us %.2f" % (d["ppo_update"]["fused_ms_per_minibatch"] * 1e3),
      "train it ms %.3f" % d["train_iteration"]["ms_per_iteration"], "%.4g env-steps/s" % d["train_iteration"]["value"])
PY
echo session done
