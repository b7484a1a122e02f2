# import-order check of the per-env drop-in classes (a fresh interpreter per case)
mkdir -p gpurun_out
timeout -k 5 120 python -c "
import sys; sys.path.insert(0,'gym-lorenz_amd')
import gym_lorenz as gl
e = gl.make('lorenz_dynamic-v0'); print('gym_lorenz-first ok', e.reset())" > gpurun_out/diag_a.txt 2>&1
echo "rc=$?" >> gpurun_out/diag_a.txt
