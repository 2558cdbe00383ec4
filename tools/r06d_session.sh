R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R" || exit 2
OUT=gpurun_out/r06d; mkdir -p $OUT
for c in 0 4 64; do
  RR_EXACT_CP_MAX=$c RR_LIB_PATH=tools/ab/lib_xstamps.so timeout -k 10 200 python tools/exact_stamps.py --n 65536 --out $OUT/stamps_cp$c.json > $OUT/stamps_cp$c.log 2>&1 || exit $?
  cat $OUT/stamps_cp$c.log
done
bash tools/ab_env.sh r06d/ab exact cp0=tree,RR_EXACT_CP_MAX=0 cp64=tree,RR_EXACT_CP_MAX=64 cp2=tree,RR_EXACT_CP_MAX=2
