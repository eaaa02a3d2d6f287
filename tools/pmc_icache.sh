#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r02_ic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A="--workload config5 --games 65536 --iterations 32 --chunk 32 --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY -d $OUT/p1 -o run --output-format csv -- python3 $R/bench.py $A > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $OUT/p2 -o run --output-format csv -- python3 $R/bench.py $A > $OUT/p2.log 2>&1 || exit 2
A3="--steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY -d $OUT/p3 -o run --output-format csv -- python3 $R/bench.py $A3 > $OUT/p3.log 2>&1 || exit 3
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $OUT/p4 -o run --output-format csv -- python3 $R/bench.py $A3 > $OUT/p4.log 2>&1 || exit 4
A5="--steps 2 --warmup 1 --no-cpu-baseline --order frontier"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY -d $OUT/p5 -o run --output-format csv -- python3 $R/bench.py $A5 > $OUT/p5.log 2>&1 || exit 5
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $OUT/p6 -o run --output-format csv -- python3 $R/bench.py $A5 > $OUT/p6.log 2>&1 || exit 6
echo done
