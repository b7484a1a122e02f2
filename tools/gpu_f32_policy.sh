set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy_edges.py tests/test_gpu_policy.py -x -q -m gpu -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pol_tests.log 2>&1 || exit $?
for cfg in "pmsm 262144 16 8192" "pmsm 32768 2048 8192" "lorenz3 1048576 16 1024"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --mode policy --system $1 --envs $2 --K $3 --steps $4 > gpurun_out/polf32_$1_$2_$3.json 2> gpurun_out/polf32_$1_$2_$3.err || exit $?
  timeout -k 10 300 python bench.py --mode policy --precision bf16 --system $1 --envs $2 --K $3 --steps $4 > gpurun_out/polbf16_$1_$2_$3.json 2> gpurun_out/polbf16_$1_$2_$3.err || exit $?
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/polf32_prof -o run --output-format csv -- python bench.py --mode policy --system pmsm --envs 262144 --K 16 --steps 2048 > gpurun_out/polf32_prof.log 2>&1
