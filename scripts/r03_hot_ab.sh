#!/bin/bash
# Stage 4's hot-key path A/B (ORL_NO_HOT=1 turns it off): its parity test, config 2 bench (no hot key: the pick's
# overhead) and the per-rank cost of config 3 at 8 ranks (the hot rank takes the path).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r03d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k hot_key --timeout 240 --timeout-method thread > $O/hot.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > $O/c2.json 2> $O/c2.log &&
ORL_NO_HOT=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > $O/c2_nohot.json 2> $O/c2_nohot.log &&
timeout -k 10 300 python -u scripts/rank_cost_lab.py 8 4 8 > $O/rank.log 2>&1 &&
ORL_NO_HOT=1 timeout -k 10 300 python -u scripts/rank_cost_lab.py 8 4 8 > $O/rank_nohot.log 2>&1
