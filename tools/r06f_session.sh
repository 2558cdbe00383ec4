#!/bin/bash
# exact mode: the component-interleaved tableau / error-norm order (tools/ab/lib_ilv.so) against the
# in-tree kernels: bitwise first (both 6DOF kernels), then timing
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT=gpurun_out/r06f; mkdir -p $OUT
timeout -k 10 300 python tools/exact_bitwise_ab.py --libs tree,tools/ab/lib_ilv.so --out $OUT/bitwise_ilv.json > $OUT/bitwise_ilv.log 2>&1 || { tail -5 $OUT/bitwise_ilv.log; exit 1; }
timeout -k 10 300 python tools/exact_bitwise_ab.py --libs tree,tools/ab/lib_ilv.so --lean --out $OUT/bitwise_ilv_lean.json > $OUT/bitwise_ilv_lean.log 2>&1 || { tail -5 $OUT/bitwise_ilv_lean.log; exit 1; }
cat $OUT/bitwise_ilv.json $OUT/bitwise_ilv_lean.json
bash tools/ab_env.sh r06f/exact_ab exact tree=tree ilv=ilv
