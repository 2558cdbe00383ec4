#!/bin/bash
# A/B of libraries and run-time settings, interleaved over two repetitions (as tools/ab_libs.sh, whose
# variants differ in the library only). A variant is NAME=LIB[,VAR=VALUE...]; LIB "tree" is the
# in-tree library, else tools/ab/lib_LIB.so.
#   tools/ab_env.sh TAG exact   cp0=cp,RR_EXACT_CP_MAX=0 cp4=cp,RR_EXACT_CP_MAX=4   (N = 65 536 and 524 288)
#   tools/ab_env.sh TAG rollout base=cp brcp=brcp                                  (collect, us per collect)
# CHECK="tests/..." runs those GPU tests once per distinct library first (exits on a failure).
TAG=${1:-ab}; MODE=${2:-exact}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
libpath() { if [ "$1" = tree ]; then echo "$R/rl_rocket_amd/librocket_hip.so"; else echo "$R/tools/ab/lib_$1.so"; fi; }
# env assignments of a variant spec as "VAR=VALUE ..." (the library first)
envs() { local spec=${1#*=}; local lib=${spec%%,*}; local rest=""; [ "$spec" != "$lib" ] && rest=${spec#*,};
  echo "RR_LIB_PATH=$(libpath "$lib") ${rest//,/ }"; }
if [ -n "$CHECK" ]; then
  for lib in $(for v in "$@"; do s=${v#*=}; echo "${s%%,*}"; done | sort -u); do
    env RR_LIB_PATH="$(libpath "$lib")" timeout -k 10 600 python -u -m pytest $CHECK -x -q --timeout 300 \
      --timeout-method thread -m gpu > "$OUT/test_$lib.log" 2>&1
    rc=$?
    echo "[test $lib] exit $rc" | tee -a "$OUT/status.txt"
    tail -2 "$OUT/test_$lib.log"
    if [ "$rc" -ne 0 ]; then tail -40 "$OUT/test_$lib.log"; exit "$rc"; fi
  done
fi
run() {  # run VARIANT REP [N]
  local name=${1%%=*}; local tag=${name}_$2${3:+_n$3}
  if [ "$MODE" = rollout ]; then
    env $(envs "$1") timeout -k 10 200 python bench.py --mode rollout --steps 320 --no-ppo \
      > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  else
    local k=200; [ "$3" -gt 65536 ] && k=50
    env $(envs "$1") timeout -k 10 200 python bench.py --integrator dopri5 --n "$3" --steps $k --warmup 10 \
      --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  fi
  local rc=$?
  echo "[$tag] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ]; then tail -20 "$OUT/$tag.err"; echo "stopping after $tag (rc=$rc)"; exit "$rc"; fi
  python -c "import json,sys; d=[json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')][-1]; v=d.get('gpu_ms_per_collect'); print(sys.argv[2], round((v if v is not None else d['roofline']['kernel_us'] / 1e3)*1e3, 2), 'us per', 'collect (events)' if v is not None else 'step (events)', '| wall', round(d.get('ms_per_step', 0) * 1e3, 2))" "$OUT/$tag.json" "$tag" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  for v in "$@"; do
    if [ "$MODE" = exact ]; then run "$v" "$rep" 65536 && run "$v" "$rep" 524288; else run "$v" "$rep"; fi
  done
done
echo done
