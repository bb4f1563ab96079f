# round 4 call AA: what the split's overflow reservation costs at C3 (tuning build, CCJ_ABLATE=64:
# no reservation atomic, timing only) against the same build without the ablation, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4aa_all.log && \
for a in 0 64 0 64; do CCJ_ABLATE=$a timeout -k 10 200 python -u tools/exp_split_c3.py --lib tuning c3 c3h0 > gpurun_out/r4aa_$a.log 2>&1 && grep split gpurun_out/r4aa_$a.log | sed "s/^/ablate=$a /" >> gpurun_out/r4aa_all.log || exit 1; done
