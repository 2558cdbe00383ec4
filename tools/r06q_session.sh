#!/bin/bash
# Exact mode's straggler deferral, built: its GPU tests, then events per step of the
# previous kernels (tools/ab/lib_old.so) against the tree with the deferral at caps 2 / 3 and off
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06q"; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_exact.py "tests/test_gpu_parity.py::test_action_soa_layout_is_bitwise_equal" \
  -x -v --timeout 300 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "$OUT/tests.log" | head -30; exit $rc; }
run() {  # run TAG N STEPS LIB [VAR=VALUE...]
  local tag=$1 n=$2 k=$3 lib=$4; shift 4
  env RR_LIB_PATH="$lib" "$@" timeout -k 10 300 python bench.py --integrator dopri5 --n $n --steps $k --warmup 5 \
    --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -20 "$OUT/$tag.err"; exit 3; }
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print(sys.argv[2], 'events us/step %.2f' % d['roofline']['kernel_us'], '| wall %.2f' % (d['ms_per_step']*1e3))
" "$OUT/$tag.json" "$tag" | tee -a "$OUT/summary.txt"
}
T="$R/rl_rocket_amd/librocket_hip.so"; O="$R/tools/ab/lib_old.so"
for rep in 1 2; do
  [ -n "$FULL" ] && run old_n65536_$rep 65536 200 $O
  [ -n "$FULL" ] && run tree_n65536_$rep 65536 200 $T
  [ -n "$FULL" ] && run leandefer_n65536_$rep 65536 200 $T RR_EXACT_LEAN_MIN_N=0
  for n in 524288 4194304; do
    k=50; [ $n -gt 524288 ] && k=10
    run old_n${n}_$rep $n $k $O
    run cap2_n${n}_$rep $n $k $T
    run cap3_n${n}_$rep $n $k $T RR_EXACT_DEFER_CAP=3
    run off_n${n}_$rep $n $k $T RR_EXACT_DEFER_CAP=-1
  done
done
echo done
