# round 5 call AT: gather_payload_cols<8> as the product's 8-column gather — the payload tests
# (C5, probe, bench), then the C5 profile (kernel trace + counters) of the product
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_c5_gpu.py tests/test_probe_gpu.py tests/test_bench_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r5at_tests.log 2>&1 && \
bash tools/profile_round.sh r5h c5 > gpurun_out/r5at_prof.log 2>&1
