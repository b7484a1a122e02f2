# bench.py contract checks on one GPU box: default line, a driver-like short run,
# the cfg5 rollout, and a 2-rank gloo rehearsal of the windowed timing.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20.json 2> gpurun_out/bench_s20.err || exit $?
timeout -k 10 200 python bench.py --mode rollout --K 2048 --envs 32768 --steps 16384 > gpurun_out/bench_cfg5_32k.json 2> gpurun_out/bench_cfg5_32k.err || exit $?
LZ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --envs 262144 > gpurun_out/bench_dist2.json 2> gpurun_out/bench_dist2.err || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_wrappers.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/wrappers.log 2>&1 || exit $?
timeout -k 10 120 python tools/frame_stack_bench.py > gpurun_out/fs_tile.json 2>&1 || exit $?
LZ_FRAME_STACK_ROWS=1 timeout -k 10 120 python tools/frame_stack_bench.py > gpurun_out/fs_rows.json 2>&1 || exit $?
