# k_route ILP A/B (lab builds): per-rank route at 8 ranks, config 2 and config 3 on one GPU
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
for v in main ilp2 ilp4; do
  if [ $v = main ]; then unset LAB_LIB; else export LAB_LIB=lab/liborleans_route_$v.so; fi
  timeout -k 10 300 python3 scripts/rank_cost_lab.py > $O/rank_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'hottest\|median' $O/rank_$v.txt | sed 's/receives.*//')"
  timeout -k 10 200 python3 scripts/ab_lib.py --config 2 --no-cpu > $O/c2_$v.txt 2>&1 || exit 1
  echo "$v c2: $(grep -h 'rank 0' $O/c2_$v.txt)"
  timeout -k 10 300 python3 scripts/ab_lib.py --config 3 --no-cpu --steps 10 > $O/c3_$v.txt 2>&1 || exit 1
  echo "$v c3: $(grep -h 'rank 0' $O/c3_$v.txt)"
done
