#!/bin/bash
# PPO learner session: tests, timings, rollout bench, PMC passes of ppo_grad_kernel.
set -o pipefail
TAG=${1:-ppo2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
O="$R/gpurun_out/$TAG"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_ppo.py tests/test_gpu_rollout.py > "$O/pytest.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 200 python tools/probe_ppo_grad.py > "$O/probe.json" 2> "$O/probe.err" || { echo "probe rc=$?"; tail "$O/probe.err"; exit 1; }
cat "$O/probe.json"
timeout -k 10 300 python bench.py --mode rollout --steps 320 > "$O/rollout.json" 2> "$O/rollout.err" || { echo "bench rc=$?"; tail -20 "$O/rollout.err"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$O/pmc1" -o pmc -- python "$R/tools/probe_ppo_grad.py" --only grad --calls 10 > "$O/pmc1.log" 2>&1 || { echo "pmc1 rc=$?"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d "$O/pmc2" -o pmc -- python "$R/tools/probe_ppo_grad.py" --only grad --calls 10 > "$O/pmc2.log" 2>&1 || { echo "pmc2 rc=$?"; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python "$R/tools/probe_ppo_grad.py" > "$O/kt.log" 2>&1 || { echo "kt rc=$?"; exit 1; }
echo done
