#!/bin/bash
# Isolated vs back-to-back launches of the step kernel, helper-wave kernel vs plain kernel at
# small N (RR_HELP_MAX_N=0 selects the plain kernel), and the plain kernel under rocprofv3.
TAG=${1:-iso}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "[$name] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
}
B="python $R/bench.py --no-cpu-baseline --no-sb3-legs"
for N in 65536 131072 262144; do
  for H in default 0; do
    if [ "$H" = 0 ]; then export RR_HELP_MAX_N=0; else unset RR_HELP_MAX_N; fi
    step iso_n${N}_h$H 200 $B --n $N --launch isolated --steps 300 --warmup 20 > "$OUT/iso_n${N}_h$H.json"
    step b2b_n${N}_h$H 200 $B --n $N --steps 20 --warmup 5 > "$OUT/b2b_n${N}_h$H.json"
    step b2b2000_n${N}_h$H 200 $B --n $N > "$OUT/b2b2000_n${N}_h$H.json"
  done
done
export TMPDIR=/tmp
export RR_HELP_MAX_N=0
mkdir -p "$OUT/rp_h0_n65536"
cd /tmp && step rp_h0 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp_h0_n65536" -o bench -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 20 --warmup 5 > "$OUT/rp_h0_n65536/bench.json"
echo done
