# round 5 call AA: the one-rank rehearsal with the local split on all CUs (auto at N = 1: no peers,
# no RCCL kernels to leave room for) against the 3/4 share, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --sharded --group 32 --no-cpu --part-share auto > gpurun_out/r5aa_auto_$i.log 2> gpurun_out/r5aa_auto_$i.err && \
  timeout -k 10 300 python -u bench.py --gpus 1 --sharded --group 32 --no-cpu --part-share on > gpurun_out/r5aa_on_$i.log 2> gpurun_out/r5aa_on_$i.err || exit 1
done
