mkdir -p gpurun_out/r02w
for BA in "--steps 20 --warmup 5" "--steps 2000 --warmup 20"; do
  timeout -k 10 400 python tools/bench_env_ab.py --rounds 5 --bench-args "$BA" "RR_LIB_PATH=/root/repo/.ab/m0.so" "RR_LIB_PATH=/root/repo/.ab/ht.so" "RR_LIB_PATH=/root/repo/.ab/ol.so" "RR_LIB_PATH=/root/repo/.ab/oe.so" > gpurun_out/r02w/ol.json 2>> gpurun_out/r02w/ol.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/r02w/ol.json')); print(d['bench_args']); [print(k[-8:], round(v['kernel_us']['median'],3), [round(x,3) for x in v['kernel_us']['runs']]) for k,v in d['settings'].items()]"
done
