#!/bin/bash
# PMC traffic of the step kernel (bench, N = 65 536) and its calibration on a kernel with the same
# memory pattern and known bytes (tools/pmc_calibrate.py): FETCH_SIZE and WRITE_SIZE in separate passes
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT="$R/gpurun_out/r06i"; mkdir -p "$OUT/step" "$OUT/probe"
export TMPDIR=/tmp
cd /tmp || exit 2
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/step/pmc_$C" -o pmc -- python "$R/bench.py" --no-cpu-baseline --no-sb3-legs --steps 256 --warmup 20 --n-sweep "" > "$OUT/step/pmc_$C.log" 2>&1 || exit $?
  timeout -k 10 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/probe/pmc_$C" -o pmc -- python "$R/tools/pmc_calibrate.py" run --k 64 > "$OUT/probe/pmc_$C.log" 2>&1 || exit $?
done
cd "$R" || exit 2
python tools/pmc_traffic.py "$OUT/step" --n 65536 --out "$OUT/pmc_traffic_n65536.json" > /dev/null || exit 1
python tools/pmc_calibrate.py parse "$OUT/probe" --step "$OUT/pmc_traffic_n65536.json" --out "$OUT/pmc_calibration_n65536.json"
