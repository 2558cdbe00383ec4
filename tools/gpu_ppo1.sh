set -o pipefail
O=gpurun_out/ppo1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_ppo.py > $O/pytest_ppo.log 2>&1 || { echo "ppo tests rc=$?"; tail -30 $O/pytest_ppo.log; exit 1; }
tail -3 $O/pytest_ppo.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_rollout.py > $O/pytest_rollout.log 2>&1 || { echo "rollout tests rc=$?"; tail -30 $O/pytest_rollout.log; exit 1; }
tail -2 $O/pytest_rollout.log
timeout -k 10 300 python bench.py --mode rollout --steps 320 > $O/rollout.json 2> $O/rollout.err || { echo "bench rc=$?"; tail -20 $O/rollout.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o ro -- python $GRAFT_REPO_ROOT/bench.py --mode rollout --steps 64 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
echo done
