set -o pipefail
O=gpurun_out/diag
mkdir -p $O
for c in "lorenz4 70001" "lorenz4 140001" "lorenz4 70004" "lorenz4 65537" "lorenz3 70001" "lorenz4 70001 0 0"; do
  echo "== $c" >> $O/diag.txt
  timeout -k 10 120 python tools/diag_rollout_steps.py $c >> $O/diag.txt 2>&1 || exit 1
done
