#!/bin/bash
# SQ counter pass for kernel diagnosis (own pass, kernel-trace only as allowed).
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --ba-calls 0 --pipeline-steps 0 --c3-steps 0 --c1-batch 0 --single-frames 0 --track-steps 0 --profile-steps 0}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/p1 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p1.log 2>&1 && echo p1 ok
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p2.log 2>&1 && echo p2 ok
