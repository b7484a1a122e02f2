#!/bin/bash
# Round 3: bench contract after the "windows until 200 ms" fix -- the contract test, the
# driver's short setting, and a 2-rank gloo rehearsal of the multi-rank window loop
set -o pipefail
O=gpurun_out/r03_bc
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_bench_contract.py > $O/t.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_s20.json 2> $O/bench_s20.err || exit 1
LZ_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --envs 262144 > $O/bench_dist2.json 2> $O/bench_dist2.err || exit 1
