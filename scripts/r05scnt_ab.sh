# stage-4 scatter stores (pairs, final keys and order, level-2 order): plain (default) vs non-temporal (lab build -DORL_LAB_SCATTER_NT)
set -o pipefail
O=gpurun_out/r05scnt; mkdir -p $O
for rep in 1 2; do
for v in main scnt; do
  if [ $v = main ]; then unset LAB_LIB; else export LAB_LIB=lab/liborleans_route_$v.so; fi
  timeout -k 10 300 python3 scripts/ab_lib.py --no-cpu --steps 10 > $O/c3_$v.txt 2>&1 || exit 1
  echo "$v c3: $(grep -h 'rank 0:' $O/c3_$v.txt)"
  timeout -k 10 200 python3 scripts/ab_lib.py --config 2 --no-cpu > $O/c2_$v.txt 2>&1 || exit 1
  echo "$v c2: $(grep -h 'rank 0:' $O/c2_$v.txt)"
done
done
