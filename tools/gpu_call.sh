# round 5 call AK: the N > 1 path (bench.py's own launcher, N rank processes on one GPU, gloo moving
# the all-to-alls) at N = 2 and 8, weak and strong, small sizes — one JSON line each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for w in 2 8; do for sc in weak strong; do
  OMP_NUM_THREADS=2 timeout -k 10 400 python -u bench.py --gpus $w --backend gloo --same-device --steps 2 --warmup 1 --no-cpu \
    --n-build-per-gpu 524288 --n-probe 3145728 --batches 3 --group 2 --scaling $sc > gpurun_out/r5ak_n${w}_${sc}.log 2> gpurun_out/r5ak_n${w}_${sc}.err || exit 1
done; done
