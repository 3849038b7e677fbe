#!/bin/bash
# Kernel traces of the 8-rank one-GPU rehearsal, this build vs the previous one (remote-flag route vs count pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/rft
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rft/cur -o trace -- python3 bench.py --local-ranks ${LR:-8} --config 3 --steps 3 --warmup 1 > gpurun_out/rft/cur.log 2>&1 || exit 1
LAB_LIB=tools/prev/lib_prev.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rft/prev -o trace -- python3 scripts/ab_lib.py --local-ranks ${LR:-8} --config 3 --steps 3 --warmup 1 > gpurun_out/rft/prev.log 2>&1 || exit 1
for v in cur prev; do echo "== $v"; python3 scripts/kstats.py gpurun_out/rft/$v | grep -E "k_route|k_host_rank|k_part_lb|k_hist_pairs|k_radix" ; grep rehearsal gpurun_out/rft/$v.log | cut -c1-70; done
