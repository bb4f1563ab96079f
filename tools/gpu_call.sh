# The current gpurun call's command (rewritten per call; every call of the round is recorded in
# tools/calls_r5.md).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && echo "no call"
