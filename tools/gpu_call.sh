# round 5 call AV: C5 gather forms on one box — product (cols, 5 WG/CU), the previous cols build
# (4 WG/CU), the quad form (tuning build, CCJ_GATHER_T=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5av c5 3 product tools/abx/libccj_gcols_lds.so tuning:CCJ_GATHER_T=0 tuning > gpurun_out/r5av_ab.log 2>&1
