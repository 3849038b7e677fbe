# round-5 end-of-session evidence: smoke, the default bench line (config 3, 256M, with its CPU baseline), its kernel
# trace, the other configs' lines, the per-rank cost at 8 ranks and the 8-rank rehearsal
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/config3_bench.txt 2>&1 || exit 1
grep -h "^{" $O/config3_bench.txt > $O/config3_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3trace -o trace -- python3 bench.py --no-cpu --steps 10 > $O/config3_trace.log 2>&1 || exit 1
python3 scripts/kstats.py $O/c3trace > $O/config3_kernel_stats.txt
for c in 2 4 5 1; do
  timeout -k 10 300 python3 bench.py --config $c > $O/config${c}_bench.txt 2>&1 || exit 1
  grep -h "^{" $O/config${c}_bench.txt > $O/config${c}_bench.json
done
timeout -k 10 300 python3 scripts/rank_cost_lab.py > $O/rank_cost_8ranks.txt 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --local-ranks 8 --no-cpu > $O/rehearsal.txt 2>&1 || exit 1
grep -h "^{" $O/rehearsal.txt > $O/node_rehearsal_8ranks_config3.json
head -8 $O/config3_kernel_stats.txt
for c in 3 2 4 5 1; do python3 -c "
import json; d=json.load(open('$O/config${c}_bench.json')); r=d.get('roofline') or {}; cb=d.get('cpu_baseline') or {}
print('config $c', round(d['ms_per_step'],4), 'ms', '%.3g'%d['value'], d['unit'], 'frac', r.get('frac'), 'cpu', cb.get('value'))"; done
grep -h "hottest\|median\|hop 1" $O/rank_cost_8ranks.txt | sed 's/receives.*//'
python3 -c "
import json; d=json.load(open('$O/node_rehearsal_8ranks_config3.json')); print('rehearsal', d['ms_per_step'], d.get('check'))"
