# k_gae schedule threshold: double-buffered for every n (ab_builds/lib_gae_db_all.so)
# vs the in-tree dispatch (double-buffered below 131,072 envs), around the threshold.
set -e
mkdir -p gpurun_out
for r in 1; do
  for sz in "131072 512" "196608 256" "262144 256" "1048576 64"; do
    LZ_LIB_AB=$PWD/ab_builds/lib_gae_db_all.so timeout -k 10 120 python tools/gae_bench.py $sz >> gpurun_out/gae_thr.jsonl
    timeout -k 10 120 python tools/gae_bench.py $sz >> gpurun_out/gae_thr.jsonl
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_policy_edges.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pol_tests.log 2>&1
