#!/bin/bash
# A/B of code generation: the same tree built into several libraries under tools/ab/
# (lib_<name>.so, via RR_LIB_PATH), each checked by the parity tests of the kernel under study and
# then timed, interleaved over two repetitions.
#   tools/ab_libs.sh TAG rollout NAME...   rollout collect (--no-ppo), us per collect
#   tools/ab_libs.sh TAG exact NAME...     exact mode at N = 65 536 and 524 288, ms per step
#   tools/ab_libs.sh TAG ppo NAME...       fused PPO minibatch update (rollout bench with PPO), ms
# The libraries are built beforehand, in this container, from edited copies of the sources, e.g.
#   python -c "from rl_rocket_amd import build as B; B.build_lib(out='tools/ab/lib_x.so', extra=[...])"
# (tools/ab/ is not committed; the A/B summaries go to profiles/rNN/ab_*/).
TAG=${1:-ab}; MODE=${2:-rollout}; shift 2
NAMES=${*:-"base"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
case "$MODE" in
  rollout) TESTS=tests/test_gpu_rollout.py ;;
  ppo) TESTS=tests/test_gpu_ppo.py ;;
  *) TESTS=tests/test_gpu_exact.py ;;
esac
chk() {  # chk NAME: parity tests against this library
  RR_LIB_PATH="$R/tools/ab/lib_$1.so" timeout -k 10 300 python -u -m pytest "$TESTS" -x -q \
    --timeout 120 --timeout-method thread -m gpu > "$OUT/test_$1.log" 2>&1
  local rc=$?
  echo "[test $1] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ]; then tail -30 "$OUT/test_$1.log"; exit "$rc"; fi
}
run() {  # run NAME REP [N]
  local tag=$1_$2${3:+_n$3}
  if [ "$MODE" = rollout ]; then
    RR_LIB_PATH="$R/tools/ab/lib_$1.so" timeout -k 10 200 python bench.py --mode rollout --steps 320 --no-ppo \
      > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  elif [ "$MODE" = ppo ]; then
    RR_LIB_PATH="$R/tools/ab/lib_$1.so" timeout -k 10 300 python bench.py --mode rollout --steps 32 \
      > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  else
    RR_LIB_PATH="$R/tools/ab/lib_$1.so" timeout -k 10 200 python bench.py --integrator dopri5 --n "$3" --steps 50 \
      --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  fi
  local rc=$?
  echo "[$tag] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ]; then echo "stopping after $tag (rc=$rc)"; exit "$rc"; fi
  python -c "import json,sys; d=[json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')][-1]; v=d.get('gpu_ms_per_collect'); u=d.get('ppo_update') or {}; print(sys.argv[2], round((v if v is not None else d['ms_per_step'])*1e3, 2), 'us per', 'collect' if v is not None else 'step', '| ppo us per minibatch', round(u.get('fused_ms_per_minibatch', 0)*1e3, 2))" "$OUT/$tag.json" "$tag" | tee -a "$OUT/summary.txt"
}
# AB_NOCHECK=1: time only (the libraries' parity was checked in the same session by other means,
# e.g. a baseline build of the previous code and the in-tree library under the GPU suite)
[ -z "$AB_NOCHECK" ] && for n in $NAMES; do chk "$n"; done
for rep in 1 2; do
  for n in $NAMES; do
    if [ "$MODE" = exact ]; then run "$n" "$rep" 65536 && run "$n" "$rep" 524288; else run "$n" "$rep"; fi
  done
done
