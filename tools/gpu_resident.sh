#!/bin/bash
# Resident step server: its tests, the drop-in class tests, then the per-env latency.
set -e
out=gpu_resident
mkdir -p gpurun_out/$out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_resident.py tests/test_gpu_parity.py -k "resident or dropin" \
  > gpurun_out/$out/tests.txt 2>&1
timeout -k 10 180 python tools/single_env_latency.py > gpurun_out/$out/latency.json 2> gpurun_out/$out/latency.err
for vb in 512 1024; do
  LZ_VN_BLOCK=$vb timeout -k 10 120 python bench.py --mode vecnorm --system pmsm --envs 262144 \
    --steps 2048 --warmup 256 > gpurun_out/$out/vn_$vb.json
done
