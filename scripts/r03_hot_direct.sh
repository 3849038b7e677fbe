#!/bin/bash
# Round 3: stage 4's hot run written straight into `order` (default) vs the scratch run + k_hot_tail copy (ORL_HOT_TAIL=1):
# parity of the hot-key path and the node, then the hot rank's per-step cost both ways and the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc"; grep -E "ms/step|passed|failed|hottest|median|Error|error" "gpurun_out/$name.log" | tail -4
  [ $rc = 0 ] || exit $rc
}
run hd_tests 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_node.py -x -v -m gpu --timeout 600 --timeout-method thread \
  -k "stage4 or config2 or unregistered or node"
run hd_rank 400 python scripts/rank_cost_lab.py 8 4 8
run hd_rank_tail 400 env ORL_HOT_TAIL=1 python scripts/rank_cost_lab.py 8 4 8
run hd_bench 120 python bench.py --steps 20 --warmup 5 --no-cpu
run hd_bench_unreg 180 python bench.py --steps 20 --warmup 5 --no-cpu --unregistered 0.1
run hd_bench_unreg_tail 180 env ORL_HOT_TAIL=1 python bench.py --steps 20 --warmup 5 --no-cpu --unregistered 0.1
