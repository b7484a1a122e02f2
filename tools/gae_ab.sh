# GAE schedule A/B on the box: lz_gae alone (tools/gae_bench.py) for an older build
# (ab_builds/lib_gae_old.so) against the in-tree library, alternated, at cfg5's per-GPU
# batch and at 262,144 envs; then the GAE parity tests.
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  for sz in "32768 2048" "262144 256" "65536 1024"; do
    LZ_LIB_AB=$PWD/ab_builds/lib_gae_old.so timeout -k 10 120 python tools/gae_bench.py $sz >> gpurun_out/gae_ab.jsonl
    timeout -k 10 120 python tools/gae_bench.py $sz >> gpurun_out/gae_ab.jsonl
  done
done
timeout -k 10 300 python -u -m pytest tests -v -m gpu -k "gae" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gae_tests.log 2>&1
timeout -k 10 300 python bench.py --mode policy --system pmsm --envs 32768 --K 2048 --steps 8192 > gpurun_out/policy_32k.log 2>&1
