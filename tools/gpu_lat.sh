# zero-copy single-env shims + exact-mode pow: GPU tests, host-latency probe, host launch cost, exact bench
O=gpurun_out/${1:-lat2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_envs.py tests/test_capi.py tests/test_gpu_exact.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --integrator dopri5 --no-cpu-baseline --no-sb3-legs --n-sweep "" > $O/bench_exact.json 2> $O/bench_exact.err || exit 1
timeout -k 10 240 python tools/probe_latency.py > $O/probe.json 2> $O/probe.err || exit 1
timeout -k 10 60 ./tools/launch_host_probe > $O/launch_host.json 2> $O/launch_host.err || exit 1
timeout -k 10 60 ./tools/launch_host_probe_pl > $O/launch_host_pl.json 2> $O/launch_host_pl.err || exit 1
cat $O/launch_host.json $O/launch_host_pl.json
python -c "import json;d=json.loads(open('$O/bench_exact.json').read().strip().splitlines()[-1]);print('exact', d['ms_per_step']*1e3, d['roofline']['kernel_us'])"
echo ok
