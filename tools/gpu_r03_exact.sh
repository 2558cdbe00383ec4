#!/bin/bash
# Exact mode (fp64 DOPRI5): parity tests, bench leg, kernel trace and SQ counters.
TAG=${1:-exact}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@"
  local rc=$?
  echo "[$name] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
}
step pytest_exact 600 python -u -m pytest tests/test_gpu_exact.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_exact.log" 2>&1
tail -2 "$OUT/pytest_exact.log"
step bench_exact 300 python "$R/bench.py" --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/bench_exact.json"
cat "$OUT/bench_exact.json"
export TMPDIR=/tmp
cd /tmp || exit 2
mkdir -p "$OUT/exact_kt"
step exact_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/exact_kt" -o bench -- python "$R/bench.py" --integrator dopri5 --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/exact_kt/bench.json" 2>&1
step exact_SQ 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d "$OUT/exact_SQ" -o pmc -- python "$R/bench.py" --integrator dopri5 --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/exact_SQ.log" 2>&1
step exact_SQ2 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_SMEM --output-format csv -d "$OUT/exact_SQ2" -o pmc -- python "$R/bench.py" --integrator dopri5 --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/exact_SQ2.log" 2>&1
cd "$R" && python tools/exact_counters.py "$OUT" --out "$OUT/exact_counters.json" > /dev/null
echo done
