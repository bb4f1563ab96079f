# round 5 call BD: gather_payload_cols' column stores plain instead of non-temporal (tuning build,
# CCJ_GATHER_ABLATE=2)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5bd c5 3 tuning tuning:CCJ_GATHER_ABLATE=2 > gpurun_out/r5bd_ab.log 2>&1
