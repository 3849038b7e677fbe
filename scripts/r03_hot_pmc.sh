#!/bin/bash
# PMC passes over the hot rank's owner route + stage 4 at 8 ranks (rank_cost_lab.py, LAB_ONLY=hottest): the owner's
# L2 hit rate and fetched bytes per message (one rocprofv3 --pmc pass per counter group, no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp LAB_ONLY=hottest
OUT=gpurun_out/hotpmc
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- python3 scripts/rank_cost_lab.py 8 4 8 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($grp) exit $rc"; [ $rc = 0 ] || exit $rc
done
python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt
grep -E "k_route|k_radix|k_seg_scatter|k_seg_count|k_hist_pairs|k_hot_tail" $OUT/pmc_summary.txt
