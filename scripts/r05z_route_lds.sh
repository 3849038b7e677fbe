# route kernel histogram LDS sized to the digit (default) vs 2^11 bins (ORL_ROUTE_LDS_FULL=1)
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
for rep in 1 2; do
for v in 0 1; do
  ORL_ROUTE_LDS_FULL=$v timeout -k 10 300 python3 bench.py --no-cpu --steps 10 > $O/c3_$v.txt 2>&1 || exit 1
  echo "full=$v c3: $(grep -h 'rank 0:' $O/c3_$v.txt)"
  ORL_ROUTE_LDS_FULL=$v timeout -k 10 200 python3 bench.py --config 2 --no-cpu > $O/c2_$v.txt 2>&1 || exit 1
  echo "full=$v c2: $(grep -h 'rank 0:' $O/c2_$v.txt)"
done
done
