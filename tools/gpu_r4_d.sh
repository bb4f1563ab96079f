# round 4 call D: kernel trace of the C3 step (is probe_chain_filt running, and for how long), the
# ordered paths after the image-order unsplit, and the split's run length vs window size (tuning
# build: 256 / 128 partitions; phases.hash_find_bucket_ms is the split)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4d_ab.log && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r4d_c3kt -o kt -- python3 bench.py --workload c3 --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/r4d_c3kt.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_probe_gpu.py tests/test_pipeline_device_gpu.py -x -q --timeout 300 --timeout-method thread -k "ordered or large_tables" > gpurun_out/r4d_ordered_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --path ordered --no-cpu --no-other --steps 6 --warmup 2 > gpurun_out/r4d_c2ord.log 2>&1 && \
for v in "CCJ_WINDOW_BITS=20" "CCJ_WINDOW_BITS=21"; do \
  env $v timeout -k 10 100 python -u bench.py --lib tuning --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4d_run.log 2>&1 || exit 1; \
  echo "$v $(tail -1 gpurun_out/r4d_run.log)" >> gpurun_out/r4d_ab.log; \
done
