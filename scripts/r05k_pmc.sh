set -o pipefail
mkdir -p gpurun_out/r05k
export TMPDIR=/tmp
O=gpurun_out/r05k
timeout -k 10 -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/rk/pmc1 -o pmc -- python3 scripts/rank_cost_lab.py > $O/rk_pmc1.log 2>&1 || exit 1
timeout -k 10 -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/rk/pmc2 -o pmc -- python3 scripts/rank_cost_lab.py > $O/rk_pmc2.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O/rk --by-grid > $O/rk_pmc_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4/trace -o trace -- python3 bench.py --config 4 --no-cpu --steps 10 > $O/c4_trace.log 2>&1 || exit 1
timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4/pmc1 -o pmc -- python3 bench.py --config 4 --no-cpu --steps 3 --warmup 1 > $O/c4_pmc1.log 2>&1 || exit 1
timeout -k 10 -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c4/pmc2 -o pmc -- python3 bench.py --config 4 --no-cpu --steps 3 --warmup 1 > $O/c4_pmc2.log 2>&1 || exit 1
timeout -k 10 -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/c4/pmc3 -o pmc -- python3 bench.py --config 4 --no-cpu --steps 3 --warmup 1 > $O/c4_pmc3.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O/c4 > $O/c4_pmc_summary.txt
grep -i "k_route\|k_fanout" $O/rk_pmc_summary.txt $O/c4_pmc_summary.txt
