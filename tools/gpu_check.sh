#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step runs under its own timeout; a crash/timeout/abort ends the script.
# Usage: tools/gpu_check.sh TAG [pytest-args...]
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
ok_or_testfail() {  # 0 = pass, 1 = test failures (still safe to continue); anything else = stop
  local rc=$1 what=$2
  echo "[$what] exit $rc" | tee -a "$OUT/status.txt"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what (rc=$rc)"; exit "$rc"; fi
}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s "$@" > "$OUT/pytest_gpu.log" 2>&1
ok_or_testfail $? pytest_gpu
tail -5 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
ok_or_testfail $? smoke
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
ok_or_testfail $? bench
cat "$OUT/bench.json"
export TMPDIR=/tmp
cd /tmp || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python "$R/bench.py" --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1
ok_or_testfail $? rocprof
find "$OUT/prof" -name '*stats*' | head
if [ -n "$PMC" ]; then
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_$C" -o pmc -- python "$R/bench.py" --no-cpu-baseline --steps 256 --warmup 20 $PMC_ARGS > "$OUT/pmc_$C.log" 2>&1
    ok_or_testfail $? pmc_$C
  done
fi
if [ -n "$SQ" ]; then
  timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmc_SQ" -o pmc -- python "$R/bench.py" --no-cpu-baseline --steps 256 --warmup 20 $PMC_ARGS > "$OUT/pmc_SQ.log" 2>&1
  ok_or_testfail $? pmc_SQ
  timeout -k 10 600 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmc_GRBM" -o pmc -- python "$R/bench.py" --no-cpu-baseline --steps 256 --warmup 20 $PMC_ARGS > "$OUT/pmc_GRBM.log" 2>&1
  ok_or_testfail $? pmc_GRBM
fi
echo done
