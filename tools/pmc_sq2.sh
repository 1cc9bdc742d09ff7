#!/bin/bash
# Issue-side SQ counters of one bench config (separate passes): instruction mix, SALU/VALU busy,
# branch count, LDS conflicts, occupancy level.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES -d $OUT/a -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/a.log 2>&1 || { echo a failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/b -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/b.log 2>&1 || { echo b failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_CYCLES -d $OUT/c -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/c.log 2>&1 || { echo c failed; exit 1; }
echo done
