#!/bin/bash
# SQ counters of the device decoders (tools/run_decode.py), one pass per counter group
set -o pipefail
OUT=gpurun_out/${1:-dec}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/run_decode.py > $OUT/trace.log 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/sq1 -o run --output-format csv -- python3 tools/run_decode.py > $OUT/sq1.log 2>&1 || { echo sq1 failed; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 tools/run_decode.py > $OUT/sq2.log 2>&1 || { echo sq2 failed; exit 1; }
python3 tools/sq_table.py $OUT/sq1 dec_ col_ > $OUT/sq.txt && python3 tools/sq_table.py $OUT/sq2 dec_ col_ >> $OUT/sq.txt && cat $OUT/sq.txt
python3 - <<PY
import csv
for r in csv.DictReader(open('gpurun_out/${1:-dec}/trace/run_kernel_stats.csv')):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
