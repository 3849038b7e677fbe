# fan-out kernel's route/act stores: plain (default) vs non-temporal (lab build); configs 4 and 5
set -o pipefail
O=gpurun_out/r05fanst; mkdir -p $O
for rep in 1 2; do
for v in main fannt; do
  if [ $v = main ]; then unset LAB_LIB; else export LAB_LIB=lab/liborleans_route_$v.so; fi
  timeout -k 10 300 python3 scripts/ab_lib.py --config 4 --no-cpu > $O/c4_$v.txt 2>&1 || exit 1
  echo "$v c4: $(grep -h 'config 4: 0' $O/c4_$v.txt)"
  timeout -k 10 200 python3 scripts/ab_lib.py --config 5 --no-cpu > $O/c5_$v.txt 2>&1 || exit 1
  echo "$v c5: $(grep -h 'eager 0' $O/c5_$v.txt)"
done
done
