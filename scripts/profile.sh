#!/bin/bash
# rocprofv3 kernel-trace summary + separate PMC passes (one pass per counter group) over bench.py.
#   BENCH_ARGS   bench arguments (default: 3 steps, 1 warmup, no CPU leg)
#   PMC_GROUPS   ';'-separated counter groups (default: the HBM-traffic groups); PMC=0 skips the PMC passes
#   OUT          output directory (default gpurun_out/prof)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu}"
echo "=== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
rc=$?; echo "trace exit $rc"; grep "rank 0" $OUT/trace.log
case $rc in 124|134|137|139) exit $rc;; esac
[ "${PMC:-1}" = "0" ] && { echo "=== done (no pmc)"; exit 0; }
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum;SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  echo "=== pmc pass $i: $grp"
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i exit $rc"; tail -1 $OUT/pmc$i.log
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt
[ -z "$PMC_GROUPS" ] && python3 scripts/make_traffic_json.py $OUT ${MSGS:-67108864} $OUT/route_kernel_pmc.json
echo "=== done"
