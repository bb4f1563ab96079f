# round 4, one call: the new tests (device chaining build, work accounting, the reference's sum
# vectors on the GPU, the chaining filter walks), the C3 and C2 bench lines, then same-box A/B of the
# split (tuning build: ablations, two workgroups per CU); each step under its own limit
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4b_ab.log && \
timeout -k 10 400 python -u -m pytest tests/test_build_gpu.py tests/test_cost_gpu.py tests/test_known_answers_gpu.py tests/test_probe_gpu.py -x -q --timeout 300 --timeout-method thread -k "not micro_bench and (chain or build or cost or reference_sum)" --durations=10 > gpurun_out/r4_new.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4_c3.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4_c2.log 2>&1 && \
for v in "CCJ_ABLATE=16" "CCJ_ABLATE=48" "CCJ_SPLIT_T=512" "CCJ_SPLIT_T=1025"; do \
  env $v timeout -k 10 100 python -u bench.py --lib tuning --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4b_run.log 2>&1 || exit 1; \
  echo "$v $(tail -1 gpurun_out/r4b_run.log)" >> gpurun_out/r4b_ab.log; \
done
