# host vec-env path: pinned fetch buffers, one round trip for the small outputs, lazy done-row map
O=gpurun_out/${1:-vh4}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_envs.py tests/test_gpu_state.py tests/test_gpu_parity.py tests/test_gpu_exact.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --n-sweep "" > $O/bench_legs_$i.json 2> $O/bench_legs_$i.err || exit 1
python -c "
import json;d=json.loads(open('$O/bench_legs_$i.json').read().strip().splitlines()[-1]);l=d['sb3_legs']
print({k:(round(v['value']/1e6,1), round(v['us_per_step'],1), {a:round(b,1) for a,b in v.get('split_us_per_step',{}).items()}) for k,v in l.items()})"
done
echo ok
