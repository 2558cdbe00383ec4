#!/bin/bash
# Exact mode, VERDICT r5 item 1 by measurement: the in-tree kernels against pass-1 / pass-2 proxies of
# the two-launch straggler deferral (tools/ab_exact_cap.py: loop capped at CAP attempts, no brentq),
# events per step at N = 65 536 (in-loop kernel), 524 288 (lean kernel) and 256 (a 4-wave launch)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06p"; mkdir -p "$OUT"
for rep in 1 2; do
  for v in tree cap2 cap1; do
    lib="$R/rl_rocket_amd/librocket_hip.so"; [ $v != tree ] && lib="$R/tools/ab/lib_$v.so"
    for n in 65536 524288 256; do
      k=200; [ $n -gt 65536 ] && k=50
      RR_LIB_PATH=$lib timeout -k 10 200 python bench.py --integrator dopri5 --n $n --steps $k --warmup 10 \
        --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/${v}_n${n}_$rep.json" 2> "$OUT/${v}_n${n}_$rep.err" || { tail -20 "$OUT/${v}_n${n}_$rep.err"; exit 3; }
      python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print(sys.argv[2], 'events us/step %.2f' % d['roofline']['kernel_us'], '| wall %.2f' % (d['ms_per_step']*1e3))
" "$OUT/${v}_n${n}_$rep.json" "${v}_n${n}_$rep" | tee -a "$OUT/summary.txt"
    done
  done
done
echo done
