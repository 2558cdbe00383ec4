#!/bin/bash
# Host-side sanitizer runs (CPU, this container): the oracle (C restatement) under gcc
# ASan + UBSan against the reference's golden rows, and librocket_hip's host / C-ABI code
# under clang ASan + UBSan (hipcc -Xarch_host; device code is not instrumented: GPU ASan is
# not available on the pool) through the CPU C-ABI tests. UB aborts (no recovery); leak
# checking is off (the Python interpreter's own allocations would be reported).
# Usage: tools/sanitize.sh [OUTDIR]     -> OUTDIR/sanitize.log (default /tmp/rr_sanitize)
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/rr_sanitize}
mkdir -p "$OUT"
LOG="$OUT/sanitize.log"
: > "$LOG"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
# 1. oracle: gcc -fsanitize=address,undefined
gcc -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all -fPIC -fopenmp -std=c11 \
    -D_GNU_SOURCE -shared -o "$OUT/librocket_oracle_san.so" "$R/oracle/rocket_oracle.c" -lm || exit 2
GASAN=$(gcc -print-file-name=libasan.so)
GUBSAN=$(gcc -print-file-name=libubsan.so)
echo "== oracle (gcc ASan+UBSan): tests/test_oracle_golden.py tests/test_params.py tests/test_nonfinite.py (CPU part)" | tee -a "$LOG"
(cd "$R" && RO_LIB_PATH="$OUT/librocket_oracle_san.so" LD_PRELOAD="$GASAN:$GUBSAN" \
    python -m pytest -v -p no:cacheprovider -m "not gpu" tests/test_oracle_golden.py tests/test_params.py tests/test_nonfinite.py 2>&1) | tee -a "$LOG" | tail -4
rc1=$?
# 2. librocket_hip host code: hipcc -Xarch_host -fsanitize=address,undefined
(cd "$R" && python -c "
from rl_rocket_amd import build as b
import subprocess
cmd = b.command(out='$OUT/librocket_hip_san.so', extra=('-Xarch_host', '-fsanitize=address', '-Xarch_host',
                '-fsanitize=undefined', '-Xarch_host', '-fno-sanitize-recover=all', '-Xarch_host', '-fno-omit-frame-pointer'))
subprocess.check_call(cmd)
") || exit 3
CASAN=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
echo "== librocket_hip host code (clang ASan+UBSan): tests/test_capi.py" | tee -a "$LOG"
(cd "$R" && RR_LIB_PATH="$OUT/librocket_hip_san.so" LD_PRELOAD="$CASAN" \
    python -m pytest -v -p no:cacheprovider tests/test_capi.py -k "not library_exports" 2>&1) | tee -a "$LOG" | tail -4
rc2=$?
echo "oracle rc=$rc1 host-abi rc=$rc2" | tee -a "$LOG"
[ $rc1 -eq 0 ] && [ $rc2 -eq 0 ]
