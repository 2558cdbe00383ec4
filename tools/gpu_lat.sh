# zero-copy single-env shims: GPU tests, host-latency probe, host launch cost per HIP entry point
O=gpurun_out/${1:-lat2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_envs.py tests/test_capi.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 240 python tools/probe_latency.py > $O/probe.json 2> $O/probe.err || exit 1
timeout -k 10 60 ./tools/launch_host_probe > $O/launch_host.json 2> $O/launch_host.err || exit 1
timeout -k 10 60 ./tools/launch_host_probe_pl > $O/launch_host_pl.json 2> $O/launch_host_pl.err || exit 1
cat $O/launch_host.json $O/launch_host_pl.json
echo ok
