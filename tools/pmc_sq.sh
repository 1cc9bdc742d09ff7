#!/bin/bash
# SQ-level counters for one bench config (separate pass per counter group).
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/sq1 -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/sq1.log 2>&1 || { echo sq1 failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/sq2.log 2>&1 || { echo sq2 failed; exit 1; }
echo done
