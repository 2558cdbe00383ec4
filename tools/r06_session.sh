#!/bin/bash
# Round-6 GPU session: the GPU suite + smoke on the in-tree library, then the A/Bs of this round's
# candidates (tools/ab_env.sh): exact mode's component-parallel stragglers (RR_EXACT_CP_MAX) against
# the previous exact kernels (tools/ab/lib_old.so), and the collect's batch-inverted reciprocals.
TAG=${1:-r06}; PHASES=${2:-"tests exact rollout"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
has() { case " $PHASES " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "[pytest_gpu] exit $rc" | tee -a "$OUT/status.txt"; tail -3 "$OUT/pytest_gpu.log"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|error" "$OUT/pytest_gpu.log" | head -20; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "[smoke] exit $rc" | tee -a "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
fi
if has exact; then
  bash tools/ab_env.sh "$TAG/exact_ab" exact old=old cp0=tree,RR_EXACT_CP_MAX=0 cp4=tree,RR_EXACT_CP_MAX=4 cp8=tree,RR_EXACT_CP_MAX=8 || exit $?
fi
if has rollout; then
  CHECK=tests/test_gpu_rollout.py bash tools/ab_env.sh "$TAG/rollout_ab" rollout base=tree brcp=brcp || exit $?
fi
echo session done
