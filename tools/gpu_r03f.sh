#!/bin/bash
# resident server (command line) tests + latency; f32 attention tests + benches with
# rocprofv3 kernel-trace summaries (the roofline's per-launch time cross-check)
set -u
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
ok() { local s=$1; [ $s -eq 0 ] || [ $s -eq 1 ] || exit $s; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_gpu_resident.py tests/test_gpu_policy_attn_f32.py -s > $O/tests.txt 2>&1; ok $?
timeout -k 10 200 python -u tools/resident_latency.py > $O/resident_latency.json 2> $O/resident_latency.log || exit 1
timeout -k 10 240 python -u tools/single_env_latency.py > $O/single_env_latency.json 2> $O/single_env_latency.log || exit 1
for P in attn attn_ln; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$P -o run -- python bench.py --mode policy --policy $P --system hr --envs 32768 --K 2048 --steps 4096 > $O/bench_$P.json 2> $O/bench_$P.log || exit 1
done
