O=gpurun_out/r02sqc; mkdir -p $O; export TMPDIR=/tmp; R=$(pwd)
cd /tmp || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ --output-format csv -d $R/$O/icache -o pmc -- python $R/bench.py --no-cpu-baseline --steps 256 --warmup 20 > $R/$O/icache.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_TC_DATA_READ_REQ --output-format csv -d $R/$O/dcache -o pmc -- python $R/bench.py --no-cpu-baseline --steps 256 --warmup 20 > $R/$O/dcache.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $R/$O/ifetch -o pmc -- python $R/bench.py --no-cpu-baseline --steps 256 --warmup 20 > $R/$O/ifetch.log 2>&1 || exit 1
cd $R && python - <<'PY'
import csv, glob, statistics, collections
for sub in ('icache','dcache','ifetch'):
    f=glob.glob('gpurun_out/r02sqc/%s/**/*counter_collection.csv'%sub, recursive=True)
    if not f: print(sub,'missing'); continue
    vals=collections.defaultdict(list)
    for row in csv.DictReader(open(f[0])):
        if 'step_kernel<6, 0, false, true, 4' not in row.get('Kernel_Name',''): continue
        vals[row['Counter_Name']].append(float(row['Counter_Value']))
    print(sub, {k: statistics.median(v) for k,v in vals.items()}, {k: len(v) for k,v in vals.items()})
PY
