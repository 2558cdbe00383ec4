# exact mode: parity tests on the library as built, then A/B against tools/ab_exact/librocket_hip.so
# (the previous exact kernel) interleaved x3 at N = 65536
O=gpurun_out/${1:-abex}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_exact.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline --n-sweep "" > $O/new_$i.json 2> $O/new_$i.err || exit 1
  RR_LIB_PATH=tools/ab_exact/librocket_hip.so timeout -k 10 120 python bench.py --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline --n-sweep "" > $O/old_$i.json 2> $O/old_$i.err || exit 1
done
python - <<PY
import json,glob
for f in sorted(glob.glob("$O/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f.split("/")[-1], round(d["roofline"]["kernel_us"],3))
PY
echo ok
