#!/bin/bash
# A/B of the rollout collect's wave layout (round 4): 64 envs per wave (default) vs 32 envs per
# wave with two waves per SIMD, the second one's start staggered by S x 127 x 64 cycles.
#   tools/ab_rollout.sh TAG
TAG=${1:-ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
run() {  # run NAME env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --mode rollout --steps 320 --no-ppo > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
  python -c "import json,sys; d=[json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')][-1]; print(sys.argv[2], round(d['gpu_ms_per_collect']*1e3, 1), 'us per collect')" "$OUT/$name.json" "$name" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  run ntw2_$rep RR_ROLLOUT_NTW=2
  for S in 0 1 2 3; do run ntw1_s${S}_$rep RR_ROLLOUT_NTW=1 RR_ROLLOUT_STAGGER=$S; done
done
