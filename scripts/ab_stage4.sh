#!/bin/bash
# A/B of the stage-4 variants on config 2 (kernel trace per variant): env pairs/soa x uniform fast path on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in "soa:ORL_STAGE4_SOA=1 ORL_RANK_UNIFORM=1" "soa_nouni:ORL_STAGE4_SOA=1 ORL_RANK_UNIFORM=0" "pairs:ORL_STAGE4_SOA=0 ORL_RANK_UNIFORM=1" "pairs_nouni:ORL_STAGE4_SOA=0 ORL_RANK_UNIFORM=0"; do
  name=${v%%:*}; envs=${v#*:}
  echo "=== $name ($envs)"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$name -o t -- python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu} > gpurun_out/ab/$name.log 2>&1
  rc=$?; grep "rank 0:" gpurun_out/ab/$name.log
  case $rc in 0) ;; *) echo "exit $rc"; exit $rc;; esac
  python3 scripts/kstats.py gpurun_out/ab/$name | grep -E "radix|seg_|route<" 
done
