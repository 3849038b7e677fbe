# config 3's k_route: what its stage-4 histogram costs (lab builds: no LDS atomics / no row store)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
for v in main noatom nostore; do
  if [ $v = main ]; then unset LAB_LIB; else export LAB_LIB=lab/liborleans_route_$v.so; fi
  LAB_C3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o rl -- python3 scripts/route_lab.py 5 > $O/$v.log 2>&1 || exit 1
  echo "$v:"; python3 scripts/kstats.py $O/$v | grep "k_route"
done
