#!/bin/bash
# the multi-rank launcher path after the sweep's per-rank rows: 2 and 4 ranks on one GPU over gloo
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06k"; mkdir -p "$OUT"
export RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_gpus2_gloo.json" 2> "$OUT/bench_gpus2_gloo.err" || exit $?
timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 > "$OUT/bench_gpus4_gloo.json" 2> "$OUT/bench_gpus4_gloo.err" || exit $?
python -c "
import json,sys
for f in sys.argv[1:]:
    d=[json.loads(l) for l in open(f) if l.startswith('{')][-1]
    print(f.split('/')[-1], d['n_gpus'], '%.3e' % d['value'], [round(r['wall_ms_per_step']*1e3,2) for r in d['per_rank']], [(s['envs_per_gpu'], round(s['per_rank_wall_max_over_min'],3)) for s in d['n_sweep']], 'gather' , d.get('allgather',{}).get('value'))
" "$OUT/bench_gpus2_gloo.json" "$OUT/bench_gpus4_gloo.json"
