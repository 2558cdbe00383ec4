O=gpurun_out/${LEGS_TAG:-r02legs}; mkdir -p $O
run() { local name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; exit 1; }; python -c "
import json; d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]); r=d.get('roofline') or {}
print('$name', round(d['value']/1e9,3), 'G', round(d['ms_per_step']*1e3,3), 'us/step', round(r.get('frac',0) or 0,4))"; }
run n524288 --n 524288 --steps 500 --warmup 20
run cfg1_3dof_euler --model 3DOF --integrator euler --n 4096
run cfg1_3dof_rk4 --model 3DOF --n 4096
run dof3_n524288 --model 3DOF --n 524288 --steps 500 --warmup 20
run dopri5 --integrator dopri5 --steps 200 --warmup 10
run rollout_fp32 --mode rollout --steps 320
run rollout_fp16x3 --mode rollout --steps 320 --policy-dtype fp16x3
run rollout_bf16 --mode rollout --steps 320 --policy-dtype bf16
run allgather_w1 --allgather --steps 2000
