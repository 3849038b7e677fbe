#!/bin/bash
# Round-6 first GPU step: the default bench at HEAD, then config 3's LSD stage 4 in two launch forms, with the main build
# and a lab build whose radix passes take tiles in dispatch order (ORL_NO_XCD_TILE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > $OUT/bench.json 2> $OUT/bench.log || { echo bench failed; tail $OUT/bench.log; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/main -o t -- python3 scripts/lsd_lab.py 6 > $OUT/main.log 2>&1 || { echo main lab failed; tail $OUT/main.log; exit 1; }
grep "per step" $OUT/main.log; python3 scripts/kstats.py $OUT/main > $OUT/main_stats.txt; head -30 $OUT/main_stats.txt
LAB_LIB=lab/liborleans_route_noxcd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/noxcd -o t -- python3 scripts/lsd_lab.py 6 bench > $OUT/noxcd.log 2>&1 || { echo noxcd lab failed; tail $OUT/noxcd.log; exit 1; }
grep "per step" $OUT/noxcd.log; python3 scripts/kstats.py $OUT/noxcd > $OUT/noxcd_stats.txt; head -30 $OUT/noxcd_stats.txt
