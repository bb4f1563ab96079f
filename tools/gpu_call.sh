# round 5 call AD: C2 at 2 / 4 / 8 MiB table windows (1024 / 512 / 256 partitions; tuning build,
# CCJ_WINDOW_BITS), interleaved 2x; then the ordered tests on the product (walk_words_out refactor)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5wb c2 2 tuning:CCJ_WINDOW_BITS=18 tuning tuning:CCJ_WINDOW_BITS=20 > gpurun_out/r5wb_ab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_probe_gpu.py -k "ordered" > gpurun_out/r5ad_tests.log 2>&1
