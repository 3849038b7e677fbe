#!/bin/bash
# Kernel traces of the hot-key path A/B: the hot rank of config 3 at 8 ranks (rank_cost_lab LAB_ONLY=hottest) and config 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03t}
mkdir -p $O
for mode in hot nohot; do
  if [ $mode = nohot ]; then export ORL_NO_HOT=1; else unset ORL_NO_HOT; fi
  LAB_ONLY=hottest timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rank_$mode -o t -- python3 scripts/rank_cost_lab.py 8 4 8 > $O/rank_$mode.log 2>&1 || exit $?
  python3 scripts/kstats.py $O/rank_$mode > $O/rank_$mode.txt || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_$mode -o t -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/c2_$mode.log 2>&1 || exit $?
  python3 scripts/kstats.py $O/c2_$mode > $O/c2_$mode.txt || exit $?
done
rm -rf $O/rank_hot $O/rank_nohot $O/c2_hot $O/c2_nohot
