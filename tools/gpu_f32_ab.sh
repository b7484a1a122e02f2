# fp32 policy kernel change: parity first, then A/B against the previous build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy_f32.py "tests/test_gpu_policy_edges.py::test_tiny_and_ragged_batches" -x -v -s -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 || exit $?
timeout -k 10 600 python tools/ab_lib.py ab_builds/f32old/libgym_lorenz_amd.so default 4 -- --mode policy --system pmsm --envs 262144 --K 16 --steps 4096 > gpurun_out/ab_f32_pmsm262k.json 2> gpurun_out/ab_f32_pmsm262k.err || exit $?
timeout -k 10 600 python tools/ab_lib.py ab_builds/f32old/libgym_lorenz_amd.so default 2 -- --mode policy --system pmsm --envs 32768 --K 2048 --steps 8192 > gpurun_out/ab_f32_pmsm32k.json 2> gpurun_out/ab_f32_pmsm32k.err || exit $?
