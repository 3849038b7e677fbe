#!/bin/bash
# Calibrate FETCH_SIZE / TCC_EA0_RDREQ against known byte counts (microbench kernels), and list gfx950 counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list exit $?"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  echo "=== pass $i: $grp"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- ./scripts/microbench.bin > $OUT/p$i.log 2>&1
  rc=$?; echo "p$i exit $rc"; tail -2 $OUT/p$i.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
echo "=== done"
