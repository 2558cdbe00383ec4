#!/bin/bash
# wall clock of the driver's protocol (K = 20, W = 5) by how the 20 launches are grouped into graphs
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT=gpurun_out/r06e; mkdir -p $OUT
for rep in 1 2 3; do
  for gs in 20 10 5 4; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --graph-steps $gs --no-cpu-baseline --no-sb3-legs --n-sweep "" > $OUT/gs${gs}_$rep.json 2> $OUT/gs${gs}_$rep.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'wall us/step %.3f events %.3f value %.3e' % (d['ms_per_step']*1e3, d['roofline']['kernel_us'], d['value']))" $OUT/gs${gs}_$rep.json gs${gs}_$rep | tee -a $OUT/summary.txt
  done
done
# exact mode: the component-interleaved tableau / error-norm order (tools/ab/lib_ilv.so) against the
# in-tree kernels: bitwise first (both 6DOF kernels), then timing
timeout -k 10 300 python tools/exact_bitwise_ab.py --libs tree,tools/ab/lib_ilv.so --out $OUT/bitwise_ilv.json > $OUT/bitwise_ilv.log 2>&1 || { tail -5 $OUT/bitwise_ilv.log; exit 1; }
timeout -k 10 300 python tools/exact_bitwise_ab.py --libs tree,tools/ab/lib_ilv.so --lean --out $OUT/bitwise_ilv_lean.json > $OUT/bitwise_ilv_lean.log 2>&1 || { tail -5 $OUT/bitwise_ilv_lean.log; exit 1; }
cat $OUT/bitwise_ilv.json $OUT/bitwise_ilv_lean.json
bash tools/ab_env.sh r06e/exact_ab exact tree=tree ilv=ilv
