# interleaved rollout-collect timing of prebuilt library variants (bench.py --mode rollout)
# usage: tools/rollout_ab.sh OUTDIR lib1.so lib2.so ...
OUT=$1; shift
mkdir -p "$OUT"
for r in 1 2 3; do
  for L in "$@"; do
    RR_LIB_PATH=$L timeout -k 10 120 python bench.py --mode rollout --steps 512 --no-cpu-baseline > "$OUT/$(basename $L .so)_$r.json" 2> "$OUT/$(basename $L .so)_$r.err" || exit 3
  done
done
