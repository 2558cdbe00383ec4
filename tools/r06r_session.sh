#!/bin/bash
# Exact-mode deferral: rocprofv3 kernel trace of the two launches at N = 524 288 (cap 2) and of the one-pass lean kernel
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06r"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in cap2 off; do
  cap=2; [ $v = cap0 ] && cap=0; [ $v = off ] && cap=-1
  RR_EXACT_DEFER_CAP=$cap timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o run -- python3 "$R/bench.py" --integrator dopri5 --n 524288 --steps 20 --warmup 5 \
    --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/$v.json" 2> "$OUT/$v.err" || { tail -20 "$OUT/$v.err"; exit 3; }
done
echo done
