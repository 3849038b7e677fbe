# the default bench line and config 2 at the round's last build, with the kernel trace of the default line
set -o pipefail
O=gpurun_out/r05w2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/config3_bench.txt 2>&1 || exit 1
grep -h "^{" $O/config3_bench.txt > $O/config3_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3trace -o trace -- python3 bench.py --no-cpu --steps 10 > $O/config3_trace.log 2>&1 || exit 1
python3 scripts/kstats.py $O/c3trace > $O/config3_kernel_stats.txt
timeout -k 10 300 python3 bench.py --config 2 > $O/config2_bench.txt 2>&1 || exit 1
grep -h "^{" $O/config2_bench.txt > $O/config2_bench.json
timeout -k 10 300 python3 scripts/rank_cost_lab.py > $O/rank_cost_8ranks.txt 2>&1 || exit 1
head -3 $O/config3_kernel_stats.txt
for c in 3 2; do python3 -c "
import json; d=json.load(open('$O/config${c}_bench.json')); r=d.get('roofline') or {}; cb=d.get('cpu_baseline') or {}
print('config $c', round(d['ms_per_step'],4), 'ms', '%.4g'%d['value'], d['unit'], 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'cpu', cb.get('value'))"; done
grep -h "hottest\|median\|hop 1" $O/rank_cost_8ranks.txt | sed 's/receives.*//'
