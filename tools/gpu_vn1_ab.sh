#!/bin/bash
# TIMING ONLY: phases of the single-launch VecNormalize step (variant bits skip parts)
set -u
export TMPDIR=/tmp
O=gpurun_out/vn1_ab
mkdir -p $O
B="python bench.py --mode vecnorm --system pmsm --envs 262144 --steps 2048 --warmup 128 --no-cpu-baseline"
for V in 0 8192 16384 24576 32768 57344; do
  LZ_BENCH_VARIANT=$V timeout -k 10 200 $B > $O/v$V.json 2> $O/v$V.log || exit 1
done
timeout -k 10 200 $B --vn-launch two > $O/two.json 2> $O/two.log || exit 1
