#!/bin/bash
# bench.py's step-only graphs: plain-HIP capture / replay (default) against torch.cuda.CUDAGraph
# (--torch-graph, whose replay launches torch's RNG prologue first), the driver's command, interleaved
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06u"; mkdir -p "$OUT"
for rep in 1 2 3; do
  for v in hip torch; do
    flag=""; [ $v = torch ] && flag="--torch-graph"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" $flag \
      > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err" || { tail -20 "$OUT/${v}_$rep.err"; exit 3; }
    python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
print(sys.argv[2], d['config'].get('graph_impl'), 'value %.3f G' % (d['value']/1e9), 'wall us %.3f' % (d['ms_per_step']*1e3), 'events us %.3f' % d['roofline']['kernel_us'])
" "$OUT/${v}_$rep.json" "${v}_$rep" | tee -a "$OUT/summary.txt"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_hip" -o b -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/prof_hip.log" 2>&1 || exit 3
echo done
