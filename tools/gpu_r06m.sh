#!/bin/bash
# r06 stage M: does the ragged full-path code (kRag) slow the whole-group rollouts? The
# product library vs an LZ_RAG=0 build (ragged groups staged), rotated rounds.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r06m
mkdir -p $O
export PYTHONUNBUFFERED=1
AB="timeout -k 10 900 python tools/ab_libs.py 3 default ablib/libgym_lorenz_amd_norag.so --"
P="--mode rollout --K 2048 --steps 8192 --no-cpu-baseline --no-drift --no-extras"
$AB $P --system pmsm --envs 32768 > $O/pmsm_pair.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
$AB $P --system pmsm --envs 32768 --variant 268435456 > $O/pmsm_onelane.json 2>> $O/ab.err || exit 1
$AB $P --system hr --envs 32768 > $O/hr.json 2>> $O/ab.err || exit 1
$AB $P --system lorenz3 --envs 32768 > $O/l3.json 2>> $O/ab.err || exit 1
for f in pmsm_pair pmsm_onelane hr l3; do python -c "
import json;d=json.load(open('$O/$f.json'))
print('$f', {k: round(sorted(v['launch_us'])[len(v['launch_us'])//2],1) for k,v in d['builds'].items()})"; done
echo done
