#!/bin/bash
# A/B of stage-4 variants (kernel trace per variant).  VARIANTS: "name:ENV=V ENV2=V;..." (default: pairs vs SoA level-2
# layout, one-digit fast path on / off); BENCH_ARGS: the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
V="${VARIANTS:-pairs:ORL_STAGE4_SOA=0 ORL_RANK_UNIFORM=1;pairs_nouni:ORL_STAGE4_SOA=0 ORL_RANK_UNIFORM=0;soa:ORL_STAGE4_SOA=1 ORL_RANK_UNIFORM=1}"
IFS=';' read -ra VS <<< "$V"
for v in "${VS[@]}"; do
  name=${v%%:*}; envs=${v#*:}
  echo "=== $name ($envs) ${BENCH_ARGS}"
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/$name -o t -- python3 bench.py ${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu} > gpurun_out/ab/$name.log 2>&1
  rc=$?; grep "rank 0:" gpurun_out/ab/$name.log
  case $rc in 0) ;; *) echo "exit $rc"; exit $rc;; esac
  python3 scripts/kstats.py gpurun_out/ab/$name | grep -E "radix|seg_|route<" 
done
