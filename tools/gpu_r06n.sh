#!/bin/bash
# r06 stage N: LZ_RAG = 2 (the product: the ragged full path for the noise-free systems only)
# vs 0 (none) vs 1 (all), whole and ragged sizes, rotated rounds; then the parity tests.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06n
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ragged.py tests/test_gpu_rollout_pair.py tests/test_gpu_parity.py -k "ragged or pair or rollout" \
  > $O/tests.txt 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error" $O/tests.txt | head; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
AB="timeout -k 10 900 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_norag.so ablib/libgym_lorenz_amd_rag1.so --"
P="--mode rollout --K 2048 --steps 8192 --no-cpu-baseline --no-drift --no-extras"
for c in "pmsm 32768" "hr 32768" "lorenz3 32768" "lorenz3 16384" "lorenz3 16400" "lorenz3 32784" "hr 32784"; do
  set -- $c
  $AB $P --system $1 --envs $2 > $O/$1_$2.json 2>> $O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/$1_$2.json'))
print('$1 $2', {k.split('_')[-1]: round(sorted(v['launch_us'])[len(v['launch_us'])//2],1) for k,v in d['builds'].items()})"
done
echo done
