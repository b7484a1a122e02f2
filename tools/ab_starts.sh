# episode-starts kernel: microbench vs the torch ops it replaced, its GPU tests, and the
# policy collect end to end (K=16 at 262,144 PMSM envs).
set -e
mkdir -p gpurun_out
timeout -k 10 120 python tools/starts_bench.py 262144 16 > gpurun_out/starts_bench.jsonl
timeout -k 10 120 python tools/starts_bench.py 32768 2048 50 >> gpurun_out/starts_bench.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_policy_edges.py tests/test_gpu_policy_attn.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pol_tests.log 2>&1
for r in 1 2 3; do timeout -k 10 200 python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 2048 --warmup 64 --no-cpu-baseline --no-drift | tail -1 >> gpurun_out/policy_262k.jsonl; done
