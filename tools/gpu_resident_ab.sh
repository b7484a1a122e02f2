#!/bin/bash
# Resident server variants: A = default build, B = ab_builds/resB, C = ab_builds/f32old
# (before the payload loads were issued together); per-env latency of each, then the
# resident tests on A and B.
set -o pipefail
O=gpurun_out/res_ab
mkdir -p $O
timeout -k 10 180 python tools/single_env_latency.py > $O/A.json 2> $O/A.err || exit 1
LZ_LIB_AB=ab_builds/resB/libgym_lorenz_amd.so timeout -k 10 180 python tools/single_env_latency.py > $O/B.json 2> $O/B.err || exit 1
LZ_LIB_AB=ab_builds/f32old/libgym_lorenz_amd.so timeout -k 10 180 python tools/single_env_latency.py > $O/C.json 2> $O/C.err || exit 1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py > $O/tests_A.txt 2>&1 || exit 1
LZ_LIB_AB=ab_builds/resB/libgym_lorenz_amd.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_resident.py > $O/tests_B.txt 2>&1 || exit 1
