# N-rank rehearsal of bench.py on ONE GPU over gloo (every rank on cuda:0): --gpus 4 and 8, the
# driver's K = 20 protocol; checks n_gpus / global_envs / world_size in each line
O=gpurun_out/${1:-ranks}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_envs.py > $O/pytest_envs.log 2>&1 || { tail -30 $O/pytest_envs.log; exit 1; }
tail -2 $O/pytest_envs.log
export RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo
for g in 4 8; do
  timeout -k 10 400 python bench.py --gpus $g --steps 20 --warmup 5 > $O/gpus${g}_gloo.json 2> $O/gpus${g}_gloo.err || { tail -20 $O/gpus${g}_gloo.err; exit 1; }
  python -c "
import json;d=json.loads([l for l in open('$O/gpus${g}_gloo.json') if l.startswith('{')][-1]);c=d['config'];a=d.get('allgather',{})
print($g, d['n_gpus'], c['global_envs'], c['world_size'], c['backend'], round(d['value']/1e9,2), 'allgather', a.get('world_size'), a.get('error'), [s['global_envs'] for s in d.get('n_sweep',[])])"
done
echo ok
