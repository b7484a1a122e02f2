#!/bin/bash
# Headline kernel (k_step LORENZ3 fp32, 1,048,576 envs): kernel-trace stats of the
# default bench command and separate FETCH_SIZE / WRITE_SIZE passes -> the
# pmc_summary.json bench.py's roofline.traffic reads.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_head
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-extras > $O/trace.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 180 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python bench.py --launch eager --steps 400 --warmup 40 --no-cpu-baseline --no-drift --no-extras > $O/$c.log 2>&1 || exit 1
done
python tools/pmc_generic.py $O/FETCH_SIZE $O/WRITE_SIZE _ZN2lz6k_stepINS_5SysL3IfEEfLi0EEEvNS_5KArgsE "k_step<lz::SysL3<float>, float, 0>" 1048576 68157440 $O/lz_step_1M_pmc_summary.json || exit 1
