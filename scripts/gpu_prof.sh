#!/bin/bash
# GPU box: HBM traffic (two separate PMC passes), the bench line, then the bench under
# rocprofv3 --kernel-trace --stats. Every GPU step has its own time limit; the script stops
# at the first failure. Outputs under gpurun_out/prof_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
SHORT="--steps 10 --warmup 3 --no-cpu --no-lm --no-c2 --no-c4 --no-rig --no-c1"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $SHORT ${PROF_ARGS} > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $SHORT ${PROF_ARGS} > $OUT/write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/write.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU -d $OUT/valu -o run --output-format csv -- python3 bench.py $SHORT ${PROF_ARGS} > $OUT/valu.log 2>&1 || { echo "valu pass failed"; tail -20 $OUT/valu.log; exit 1; }
python3 scripts/traffic.py $OUT/fetch $OUT/write profiles/traffic_latest.json --valu-dir $OUT/valu --lib deeparc-sfm_amd/libdab.so > $OUT/traffic.txt 2>&1 || { cat $OUT/traffic.txt; exit 1; }
cp profiles/traffic_latest.json $OUT/  # copy it back into profiles/ here (only gpurun_out/ returns)
head -25 $OUT/traffic.txt
timeout -k 10 600 python3 bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --no-c2 ${PROF_ARGS} > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -30 $OUT/kernel_stats.csv
