set -e
mkdir -p gpurun_out
timeout -k 10 500 python tools/ab_lib.py ab_builds/lib_mom_old.so default 4 -- --mode policy --system pmsm --envs 262144 --K 16 --steps 2048 --warmup 64 --no-cpu-baseline --no-drift > gpurun_out/ab_mom.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_policy_edges.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pol_tests.log 2>&1
