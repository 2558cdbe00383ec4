#!/bin/bash
# One GPU session of the round (phases in one gpurun call). Every GPU step has its own timeout;
# a crash / timeout / abort ends the script (exit codes other than 0 / 1 stop it).
#   tools/gpu_session.sh TAG "PHASES"   PHASES: any of tests bench dist prof pmc rollout legs floor exact exactpmc
#   (default: tests bench prof pmc rollout)
TAG=${1:-run}
PHASES=${2:-"tests bench prof pmc rollout"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {  # step NAME TIMEOUT cmd...: 0 = ok, 1 = test failures (continue), anything else = stop
  local name=$1 to=$2; shift 2
  echo "[$name] start $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "[$name] exit $rc" >> "$OUT/status.txt"; echo "[$name] exit $rc" >&2
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
}
has() { case " $PHASES " in *" $1 "*) return 0;; esac; return 1; }
python -c "import rl_rocket_amd.build as b; print(b.source_hash())" > "$OUT/source_hash.txt"
B="python $R/bench.py"
if has tests; then
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
if has bench; then
  # the driver's protocol, with the CPU baselines and the SB3-facing legs
  step bench_k20_1 500 $B --steps 20 --warmup 5 > "$OUT/bench_k20_1.json" 2> "$OUT/bench_k20_1.err"
  cat "$OUT/bench_k20_1.json"
  step bench_k20_2 300 $B --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs > "$OUT/bench_k20_2.json" 2> "$OUT/bench_k20_2.err"
  step bench_k2000 300 $B --no-cpu-baseline --no-sb3-legs > "$OUT/bench_k2000.json" 2> "$OUT/bench_k2000.err"
fi
if has dist; then
  (export RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo; step bench_gpus2_gloo 400 $B --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_gpus2_gloo.json" 2> "$OUT/bench_gpus2_gloo.err") || exit $?
  cat "$OUT/bench_gpus2_gloo.json"
  # configs[3]'s launcher path at 4 ranks: the line's per_rank rows (every rank's wall / events figure)
  (export RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo; step bench_gpus4_gloo 400 $B --gpus 4 --steps 20 --warmup 5 > "$OUT/bench_gpus4_gloo.json" 2> "$OUT/bench_gpus4_gloo.err") || exit $?
  step bench_gather_w1 300 $B --gather-leg --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs > "$OUT/bench_gather_w1.json" 2> "$OUT/bench_gather_w1.err"
fi
export TMPDIR=/tmp
if has prof; then
  # the driver's command under rocprofv3 --kernel-trace --stats (K = 20, N = 65536 and the sweep N)
  for N in 65536 524288 4194304; do
    mkdir -p "$OUT/rp_k20_n$N"
    # the sweep points at their steady state (bench.py SWEEP_MIN_WARMUP), the headline N as the driver runs it
    W=5; [ "$N" -gt 65536 ] && W=100
    (cd /tmp && step rp_n$N 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp_k20_n$N" -o bench -- python "$R/bench.py" --n $N --steps 20 --warmup $W --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/rp_k20_n$N/bench.json" 2> "$OUT/rp_k20_n$N/bench.err") || exit $?
    python tools/rocprof_step.py "$OUT/rp_k20_n$N" --out "$OUT/rocprof_step_k20_n$N.json" > /dev/null
  done
fi
if has pmc; then
  cd /tmp || exit 2
  step pmc_SQ 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc_SQ" -o pmc -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 256 --warmup 20 --n-sweep "" > "$OUT/pmc_SQ.log" 2>&1
  step pmc_SQ2 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --output-format csv -d "$OUT/pmc_SQ2" -o pmc -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 256 --warmup 20 --n-sweep "" > "$OUT/pmc_SQ2.log" 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc_$C 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 256 --warmup 20 --n-sweep "" > "$OUT/pmc_$C.log" 2>&1
  done
  cd "$R" || exit 2
  python tools/pmc_traffic.py "$OUT" --n 65536 --out "$OUT/pmc_traffic_n65536.json" > /dev/null
  python tools/sq_summary.py "$OUT" --out "$OUT/sq_counters.json" > /dev/null
fi
if has rollout; then
  # configs[4]: the collect rate + its roofline, the collect kernel under the tracer and its SQ counters
  step rollout 400 $B --mode rollout --steps 320 > "$OUT/rollout.json" 2> "$OUT/rollout.err"
  cat "$OUT/rollout.json" | head -c 600; echo
  mkdir -p "$OUT/rp_rollout"
  (cd /tmp && step rp_rollout 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp_rollout" -o bench -- python "$R/bench.py" --mode rollout --steps 320 > "$OUT/rp_rollout/bench.json" 2> "$OUT/rp_rollout/bench.err") || exit $?
  python tools/rocprof_step.py "$OUT/rp_rollout" --out "$OUT/rocprof_rollout_n65536_t16_fp32.json" > /dev/null
  cd /tmp || exit 2
  step rollout_SQ 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d "$OUT/rollout_SQ" -o pmc -- python "$R/bench.py" --mode rollout --steps 64 --no-ppo > "$OUT/rollout_SQ.log" 2>&1
  cd "$R" || exit 2
fi
if has legs; then
  # the other configurations: configs[1] (3DOF Euler, N = 4096), 3DOF RK4 at 524288, the rollout's
  # faster tower precisions
  step legs_cfg1 300 $B --model 3DOF --integrator euler --n 4096 --steps 20 --warmup 5 --no-cpu-baseline --n-sweep "" > "$OUT/legs_cfg1_3dof_euler_n4096.json" 2> "$OUT/legs_cfg1.err"
  step legs_3dof_rk4 300 $B --model 3DOF --n 524288 --steps 20 --warmup 5 --no-cpu-baseline --n-sweep "" > "$OUT/legs_3dof_rk4_n524288.json" 2> "$OUT/legs_3dof.err"
  for P in fp16x3 bf16; do
    step legs_rollout_$P 300 $B --mode rollout --steps 320 --policy-dtype $P --no-ppo > "$OUT/legs_rollout_$P.json" 2> "$OUT/legs_rollout_$P.err"
  done
fi
if has floor; then
  # the per-wave latency floor of the N = 65536 step kernel: probe kernels of its shape and memory
  # pattern + the step itself, by events (back to back) and under the kernel tracer
  step floor_ev 300 python tools/floor_probe.py run --graph --out "$OUT/floor_events.json" > "$OUT/floor_events.log" 2>&1
  mkdir -p "$OUT/floor_rp"
  (cd /tmp && step floor_rp 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/floor_rp" -o fp -- python "$R/tools/floor_probe.py" run --reps 25 > "$OUT/floor_rp/run.log" 2>&1) || exit $?
fi
if has exact; then
  step bench_exact 300 $B --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline --n-sweep "" > "$OUT/bench_exact.json" 2> "$OUT/bench_exact.err"
  cat "$OUT/bench_exact.json"
  for N in 65536 524288; do
    mkdir -p "$OUT/exact_kt_n$N"
    (cd /tmp && step exact_kt_n$N 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/exact_kt_n$N" -o bench -- python "$R/bench.py" --integrator dopri5 --n $N --steps 50 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/exact_kt_n$N/bench.json" 2>&1) || exit $?
  done
fi
if has exactpmc; then
  # the exact kernels' fp64 VALU counters at N = 65 536 (in-loop kernel) and 524 288 (lean kernel):
  # tools/exact_counters.py -> achieved fp64 FLOP/s against the 78.6 TF vector peak
  for N in 65536 524288; do
    D="$OUT/exactpmc_n$N"; mkdir -p "$D"
    step exactpmc_bench_n$N 300 $B --integrator dopri5 --n $N --steps 50 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$D/bench_exact.json" 2> "$D/bench_exact.err"
    cd /tmp || exit 2
    step exactpmc_kt_n$N 300 rocprofv3 --kernel-trace --output-format csv -d "$D/exact_kt" -o kt -- python "$R/bench.py" --integrator dopri5 --n $N --steps 50 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$D/exact_kt.log" 2>&1
    step exactpmc_sq_n$N 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$D/exact_SQ" -o pmc -- python "$R/bench.py" --integrator dopri5 --n $N --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$D/exact_SQ.log" 2>&1
    step exactpmc_sq2_n$N 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$D/exact_SQ2" -o pmc -- python "$R/bench.py" --integrator dopri5 --n $N --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$D/exact_SQ2.log" 2>&1
    cd "$R" || exit 2
    python tools/exact_counters.py "$D" --out "$OUT/exact_counters_n$N.json" > /dev/null
  done
fi
echo done
