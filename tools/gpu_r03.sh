#!/bin/bash
# Round-3 GPU session. Every GPU step has its own timeout; a crash / timeout / abort ends the
# script (exit codes other than 0 / 1 stop it).
#   tools/gpu_r03.sh TAG PHASES      PHASES: any of tests bench dist prof pmc exact (default: all)
TAG=${1:-run}
PHASES=${2:-"tests bench dist prof pmc exact"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {  # step NAME TIMEOUT cmd...: 0 = ok, 1 = test failures (continue), anything else = stop
  local name=$1 to=$2; shift 2
  echo "[$name] start $(date +%T)" >&2
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "[$name] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
}
has() { case " $PHASES " in *" $1 "*) return 0;; esac; return 1; }
python -c "import rl_rocket_amd.build as b; print(b.source_hash())" > "$OUT/source_hash.txt"
if has tests; then
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
if has bench; then
  # the driver's protocol, with the CPU baseline and the SB3-facing legs
  step bench_k20_1 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_k20_1.json" 2> "$OUT/bench_k20_1.err"
  cat "$OUT/bench_k20_1.json"
  for i in 2 3; do
    step bench_k20_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs > "$OUT/bench_k20_$i.json" 2> "$OUT/bench_k20_$i.err"
  done
  step bench_k2000 300 python bench.py --no-cpu-baseline --no-sb3-legs > "$OUT/bench_k2000.json" 2> "$OUT/bench_k2000.err"
fi
if has dist; then
  # N > 1 ranks rehearsed on one GPU (gloo), the step + all_gather leg at world 1 over RCCL, and the
  # sharded-step == one-batch check under torchrun
  (export RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo; step bench_gpus2_gloo 400 python bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_gpus2_gloo.json" 2> "$OUT/bench_gpus2_gloo.err") || exit $?
  cat "$OUT/bench_gpus2_gloo.json"
  # without the rehearsal knobs on a one-GPU box: must fail loudly (exit 2, no line), before any GPU use
  timeout -k 10 120 python bench.py --gpus 2 --steps 20 --warmup 5 > "$OUT/bench_gpus2_plain.json" 2> "$OUT/bench_gpus2_plain.err"
  echo "[bench_gpus2_plain] exit $? (expected 2)" | tee -a "$OUT/status.txt"
  step bench_gather_w1 300 python bench.py --gather-leg --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs > "$OUT/bench_gather_w1.json" 2> "$OUT/bench_gather_w1.err"
  (export RR_BENCH_ONE_DEVICE=1 RR_BENCH_BACKEND=gloo; step dist_check_gloo2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 tools/dist_check.py > "$OUT/dist_check_gloo2.json" 2> "$OUT/dist_check_gloo2.err") || exit $?
  cat "$OUT/dist_check_gloo2.json"
fi
export TMPDIR=/tmp
if has prof; then
  # events vs rocprofv3 kernel-trace at four N, the driver's K = 20 protocol (+ K = 2000 at 65536)
  for N in 65536 131072 262144 524288; do
    step ev_n$N 300 python "$R/bench.py" --n $N --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs > "$OUT/ev_k20_n$N.json" 2> "$OUT/ev_k20_n$N.err"
    mkdir -p "$OUT/rp_k20_n$N"
    (cd /tmp && step rp_n$N 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp_k20_n$N" -o bench -- python "$R/bench.py" --n $N --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs > "$OUT/rp_k20_n$N/bench.json" 2> "$OUT/rp_k20_n$N/bench.err") || exit $?
    python tools/rocprof_step.py "$OUT/rp_k20_n$N" --out "$OUT/rocprof_step_k20_n$N.json" > /dev/null
  done
  mkdir -p "$OUT/rp_k2000_n65536"
  (cd /tmp && step rp_k2000 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp_k2000_n65536" -o bench -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs > "$OUT/rp_k2000_n65536/bench.json" 2> "$OUT/rp_k2000_n65536/bench.err") || exit $?
  python tools/rocprof_step.py "$OUT/rp_k2000_n65536" --out "$OUT/rocprof_step_k2000_n65536.json" > /dev/null
fi
if has pmc; then
  cd /tmp || exit 2
  step pmc_SQ 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc_SQ" -o pmc -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 256 --warmup 20 > "$OUT/pmc_SQ.log" 2>&1
  step pmc_SQ2 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --output-format csv -d "$OUT/pmc_SQ2" -o pmc -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 256 --warmup 20 > "$OUT/pmc_SQ2.log" 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc_$C 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 256 --warmup 20 > "$OUT/pmc_$C.log" 2>&1
  done
  cd "$R" || exit 2
  python tools/pmc_traffic.py "$OUT" --n 65536 --out "$OUT/pmc_traffic_n65536.json" > /dev/null
  python tools/sq_summary.py "$OUT" --out "$OUT/sq_counters.json" > /dev/null
fi
if has exact; then
  # exact mode (fp64 DOPRI5 + brentq): wall clock, kernel trace and SQ counters of step_exact_kernel
  step bench_exact 300 python "$R/bench.py" --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline --n-sweep "" > "$OUT/bench_exact.json" 2> "$OUT/bench_exact.err"
  cat "$OUT/bench_exact.json"
  cd /tmp || exit 2
  mkdir -p "$OUT/exact_kt"
  step exact_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/exact_kt" -o bench -- python "$R/bench.py" --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline --n-sweep "" > "$OUT/exact_kt/bench.json" 2>&1
  step exact_SQ 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d "$OUT/exact_SQ" -o pmc -- python "$R/bench.py" --integrator dopri5 --steps 50 --warmup 5 --no-cpu-baseline --n-sweep "" > "$OUT/exact_SQ.log" 2>&1
  step exact_SQ2 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM --output-format csv -d "$OUT/exact_SQ2" -o pmc -- python "$R/bench.py" --integrator dopri5 --steps 50 --warmup 5 --no-cpu-baseline --n-sweep "" > "$OUT/exact_SQ2.log" 2>&1
  cd "$R" || exit 2
fi
echo done
