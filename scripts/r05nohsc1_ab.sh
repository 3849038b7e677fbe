# node owner route (k_route<0>, no histogram): non-temporal stores (default) vs sc1 write-through (lab build); rank lab
set -o pipefail
O=gpurun_out/r05nohsc1; mkdir -p $O
for rep in 1 2; do
for v in main nohsc1; do
  if [ $v = main ]; then unset LAB_LIB; else export LAB_LIB=lab/liborleans_route_$v.so; fi
  timeout -k 10 300 python3 scripts/rank_cost_lab.py > $O/rank_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -h 'hottest\|median' $O/rank_$v.txt | sed 's/receives.*//' | tr '\n' ' ')"
done
done
