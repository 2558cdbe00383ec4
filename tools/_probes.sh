O=gpurun_out/r02v2; mkdir -p $O/n4m
timeout -k 10 120 python tools/hbm_probe.py > $O/hbm_probe.json 2> $O/hbm_probe.err && cat $O/hbm_probe.json && for i in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu-baseline --n 4194304 --steps 500 --warmup 20 > $O/bench_n4194304_$i.json 2> $O/bench_n4194304_$i.err || exit 1; done && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_k20.json 2> $O/bench_k20.err && timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_k2000.json 2> $O/bench_k2000.err && python -c "
import json,glob
for f in sorted(glob.glob('$O/bench_*.json')):
    d=json.loads([l for l in open(f) if l.startswith('{')][-1]); print(f, round(d['roofline']['kernel_us'],3), round(d['roofline']['frac'],4))
"
