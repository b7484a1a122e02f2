#!/bin/bash
# fp32 policy rollout: 4 vs 8 waves per workgroup at 262,144 envs (PMSM 8-wave variant
# spills 80 B/lane), and HR / LORENZ3 for comparison.
set -e
out=gpurun_out/f32_waves
mkdir -p $out
for sys in pmsm hr lorenz3; do
  for w in 4 8; do
    LZ_POL_F32_WAVES=$w timeout -k 10 200 python bench.py --mode policy --system $sys --envs 262144 \
      --K 16 --steps 4096 --no-extras > $out/${sys}_w$w.json 2> $out/${sys}_w$w.err
  done
done
