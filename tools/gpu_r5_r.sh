# round 5 call R: does loading the split's keys as 16-byte pairs lower its pattern floor?
# tools/runstore pref (8-byte loads) vs pref16, interleaved 3x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
o=gpurun_out/r5r_runstore16.log && : > $o && \
for i in 1 2 3; do
  timeout -k 10 60 ./tools/runstore 22 1 pref >> $o 2>&1 && timeout -k 10 60 ./tools/runstore 22 1 pref16 >> $o 2>&1 || exit 1
done
