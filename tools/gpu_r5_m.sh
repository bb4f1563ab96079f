# round 5 call M: owner split ablations (reservation atomics, image scatter) and the 1024-thread form
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
OWNER_TAG=r5m2 bash tools/gpu_r5_l.sh
