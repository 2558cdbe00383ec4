#!/bin/bash
# rocprofv3 kernel-trace of the step kernel for each library given (diagnostics):
#   tools/rocprof_ab.sh TAG lib1.so [lib2.so ...]
# Each run: diag_kernel child (HIP events around graph replays) under rocprofv3, so the
# profiler's per-dispatch durations and the events' per-launch period come from the same run.
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
for LIB in "$@"; do
  NAME=$(basename "$LIB" .so)
  OUT="$R/gpurun_out/$TAG/$NAME"
  mkdir -p "$OUT"
  cd /tmp || exit 2
  RR_LIB_PATH="$R/$LIB" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o rp -- python3 "$R/tools/diag_kernel.py" --child --n 65536 --model 6 --steps 1024 > "$OUT/child.log" 2>&1
  rc=$?
  echo "$NAME rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  grep '^{' "$OUT/child.log" | tail -1
  grep step_kernel "$OUT"/*kernel_stats.csv | cut -d, -f2-8 | head -2
done
