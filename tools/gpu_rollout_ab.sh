# Rollout kernel change: parity first, then A/B against the previous build
# (ab_builds/old/libgym_lorenz_amd.so) on cfg5's 32,768-env K=2048 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cfg5.py "tests/test_gpu_parity.py::test_rollout_equals_steps" "tests/test_gpu_parity.py::test_rollout_split_lanes_bitexact" -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/rollout_tests.log 2>&1 || exit $?
timeout -k 10 600 python tools/ab_lib.py ab_builds/old/libgym_lorenz_amd.so default 6 -- --mode rollout --K 2048 --envs 32768 --steps 16384 > gpurun_out/ab_rollout_32k.json 2> gpurun_out/ab_rollout_32k.err || exit $?
