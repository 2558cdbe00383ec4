# SB3 host leg: default HSA signal waits vs polling (HSA_ENABLE_INTERRUPT=0), two runs each
O=gpurun_out/vh3; mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/default_$i.json 2> $O/default_$i.err || exit 1
HSA_ENABLE_INTERRUPT=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/poll_$i.json 2> $O/poll_$i.err || exit 1
done
echo ok
