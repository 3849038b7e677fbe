# config 3's k_route with (k_route<11>) and without (k_route<0>) the stage-4 histogram: SQ instruction / cycle counters
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
LAB_C3=1 timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc1 -o pmc -- python3 scripts/route_lab.py 2 > $O/pmc1.log 2>&1 || exit 1
LAB_C3=1 timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD --output-format csv -d $O/pmc2 -o pmc -- python3 scripts/route_lab.py 2 > $O/pmc2.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O | grep "k_route"
