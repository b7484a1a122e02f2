#!/bin/bash
# Same-box A/B of the VecNormalize step: the round-2 start build (3 launches) vs HEAD,
# after the vecnorm parity tests.
set -o pipefail
O=gpurun_out/vn_abold
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vecnorm.py > $O/tests.txt 2>&1 || exit 1
for cfg in "pmsm 262144 2048" "pmsm 393216 1024" "pmsm 524288 1024" "pmsm 1048576 512" "lorenz3 1048576 512"; do
  set -- $cfg
  timeout -k 10 600 python tools/ab_lib.py ab_builds/vnold/libgym_lorenz_amd.so default 3 -- --mode vecnorm --system $1 --envs $2 --steps $3 --warmup 64 > $O/${1}_$2.json 2> $O/${1}_$2.err || exit 1
done
