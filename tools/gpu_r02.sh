#!/bin/bash
# One GPU session (round 2 protocol): parity tests, smoke, the driver's bench protocol
# (--steps 20 --warmup 5) plus the long form, rocprofv3 kernel-trace stats of the driver's
# command, SQ issue counters and HBM traffic counters in their own passes.
# Every GPU step has its own timeout; a crash / timeout / abort ends the script.
# Usage: tools/gpu_r02.sh TAG      env: TESTS=0 skips pytest, PMC=0 skips counter passes,
#                                       BENCH_ARGS="..." extra bench.py args for every bench leg
TAG=${1:-run}
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
git -C "$R" rev-parse HEAD > "$OUT/head.txt" 2>/dev/null || true
if [ "${TESTS:-1}" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
for i in 1 2 3 4 5 6; do
  step bench_k20_$i 300 python bench.py --steps 20 --warmup 5 $BENCH_ARGS > "$OUT/bench_k20_$i.json" 2> "$OUT/bench_k20_$i.err"
  cat "$OUT/bench_k20_$i.json"
done
# the same protocol on hipGraph replays (the default launch above is direct below K = 32)
for i in 1 2; do
  step bench_graph_k20_$i 300 python bench.py --no-cpu-baseline --launch graph --steps 20 --warmup 5 $BENCH_ARGS > "$OUT/bench_graph_k20_$i.json" 2> "$OUT/bench_graph_k20_$i.err"
done
step bench_k2000 300 python bench.py --no-cpu-baseline $BENCH_ARGS > "$OUT/bench_k2000.json" 2> "$OUT/bench_k2000.err"
cat "$OUT/bench_k2000.json"
# the drop-in default configuration (RocketVecEnv monitor=True: Monitor return plane per step)
step bench_monitor_k20 300 python bench.py --no-cpu-baseline --monitor --steps 20 --warmup 5 > "$OUT/bench_monitor_k20.json" 2> "$OUT/bench_monitor_k20.err"
step bench_monitor_k2000 300 python bench.py --no-cpu-baseline --monitor > "$OUT/bench_monitor_k2000.json" 2> "$OUT/bench_monitor_k2000.err"
export TMPDIR=/tmp
cd /tmp || exit 2
step rocprof_k20 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_k20" -o bench -- python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS > "$OUT/prof_k20.log" 2>&1
step rocprof_k2000 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_k2000" -o bench -- python "$R/bench.py" --no-cpu-baseline $BENCH_ARGS > "$OUT/prof_k2000.log" 2>&1
# isolated dispatches (direct launches, host-paced): kernel-trace durations without the
# profiler's back-to-back completion handling inside them
step rocprof_loop 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_loop" -o bench -- python "$R/bench.py" --no-cpu-baseline --launch loop --steps 2000 --warmup 20 $BENCH_ARGS > "$OUT/prof_loop.log" 2>&1
if [ "${PMC:-1}" = 1 ]; then
  step pmc_SQ 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc_SQ" -o pmc -- python "$R/bench.py" --no-cpu-baseline --steps 256 --warmup 20 $BENCH_ARGS > "$OUT/pmc_SQ.log" 2>&1
  step pmc_SQ2 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --output-format csv -d "$OUT/pmc_SQ2" -o pmc -- python "$R/bench.py" --no-cpu-baseline --steps 256 --warmup 20 $BENCH_ARGS > "$OUT/pmc_SQ2.log" 2>&1
  step pmc_GRBM 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_GRBM" -o pmc -- python "$R/bench.py" --no-cpu-baseline --steps 256 --warmup 20 $BENCH_ARGS > "$OUT/pmc_GRBM.log" 2>&1
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc_$C 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- python "$R/bench.py" --no-cpu-baseline --steps 256 --warmup 20 $BENCH_ARGS > "$OUT/pmc_$C.log" 2>&1
  done
  (cd "$R" && python tools/pmc_traffic.py "$OUT" --n 65536 --out "$OUT/pmc_traffic_n65536.json" > /dev/null)
  python "$R/tools/sq_summary.py" "$OUT" --out "$OUT/sq_counters.json" > /dev/null
fi
if [ "${PMC4M:-0}" = 1 ]; then  # the true-HBM point: 4 194 304 envs (> 256 MiB MALL)
  mkdir -p "$OUT/n4m"
  step hbm_probe 120 python "$R/tools/hbm_probe.py" > "$OUT/hbm_probe.json" 2> "$OUT/hbm_probe.err"
  cat "$OUT/hbm_probe.json"
  for C in FETCH_SIZE WRITE_SIZE; do
    step pmc4m_$C 180 rocprofv3 --pmc $C --output-format csv -d "$OUT/n4m/pmc_$C" -o pmc -- python "$R/bench.py" --no-cpu-baseline --n 4194304 --steps 64 --warmup 8 > "$OUT/n4m/pmc_$C.log" 2>&1
  done
  (cd "$R" && python tools/pmc_traffic.py "$OUT/n4m" --n 4194304 --out "$OUT/pmc_traffic_n4194304.json" > /dev/null)
  for i in 1 2 3; do
    step bench4m_$i 200 python "$R/bench.py" --no-cpu-baseline --n 4194304 --steps 500 --warmup 20 > "$OUT/bench_n4194304_$i.json" 2> "$OUT/bench_n4194304_$i.err"
  done
fi
echo done
