# A/B: the library as built (kernarg preload of the step kernel's first 4 arguments) against the same
# source built without preload (tools/ab_nopl/librocket_hip.so): the driver's K = 20 protocol
# interleaved x4, K = 2000 graphs x2, and the host time of one rr_step call (tools/probe_latency.py)
O=gpurun_out/${1:-abpl}; mkdir -p $O
B="--no-cpu-baseline --no-sb3-legs --n-sweep ''"
for i in 1 2 3 4; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > $O/pl_k20_$i.json 2> $O/pl_k20_$i.err || exit 1
  RR_LIB_PATH=tools/ab_nopl/librocket_hip.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > $O/nopl_k20_$i.json 2> $O/nopl_k20_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --no-sb3-legs --n-sweep "" > $O/pl_k2000_$i.json 2> $O/pl_k2000_$i.err || exit 1
  RR_LIB_PATH=tools/ab_nopl/librocket_hip.so timeout -k 10 120 python bench.py --steps 2000 --warmup 50 --no-cpu-baseline --no-sb3-legs --n-sweep "" > $O/nopl_k2000_$i.json 2> $O/nopl_k2000_$i.err || exit 1
done
python - <<PY
import json,glob
for f in sorted(glob.glob("$O/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d["roofline"]
    print(f.split("/")[-1], "events %.3f us  wall %.3f us  frac %.3f  frac_wall %.3f  G %.2f" % (r["kernel_us"], d["ms_per_step"]*1e3, r["frac"], r["frac_wall"], d["value"]/1e9))
PY
echo ok
