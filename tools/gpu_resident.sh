#!/bin/bash
# resident step server: GPU tests + latency vs number of live handles + drop-in table
set -u
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s; }
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_resident.py tests/test_gpu_rccl.py -s > $O/tests_resident.txt 2>&1; ok $?
timeout -k 10 200 python -u tools/resident_latency.py > $O/resident_latency.json 2> $O/resident_latency.log || exit 1
timeout -k 10 240 python -u tools/single_env_latency.py > $O/single_env_latency.json 2> $O/single_env_latency.log || exit 1
