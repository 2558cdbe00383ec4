#!/bin/bash
# One rocprofv3 --kernel-trace --stats sample of the driver's headline command (K = 20 graph replays,
# N = 65 536) and of the rollout collect, on whatever box this runs: committed samples make the
# median bench.py quotes (profiles/rNN/<tag>/).   tools/prof_headline.sh TAG
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT/rp_k20_n65536" "$OUT/rp_rollout"
python -c "import rl_rocket_amd.build as b; print(b.source_hash())" > "$OUT/source_hash.txt"
export TMPDIR=/tmp
cd /tmp || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp_k20_n65536" -o bench -- python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > "$OUT/rp_k20_n65536/bench.json" 2> "$OUT/rp_k20_n65536/bench.err"
rc=$?; echo "[rp_n65536] exit $rc" | tee -a "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rp_rollout" -o bench -- python "$R/bench.py" --mode rollout --steps 320 --no-ppo > "$OUT/rp_rollout/bench.json" 2> "$OUT/rp_rollout/bench.err"
rc=$?; echo "[rp_rollout] exit $rc" | tee -a "$OUT/status.txt"; [ $rc -ne 0 ] && exit $rc
cd "$R" || exit 2
python tools/rocprof_step.py "$OUT/rp_k20_n65536" --out "$OUT/rocprof_step_k20_n65536.json" | grep -E '"mean_ns"|"frac"'
python tools/rocprof_step.py "$OUT/rp_rollout" --out "$OUT/rocprof_rollout_n65536_t16_fp32.json" | grep -E '"mean_ns"|"frac"'
