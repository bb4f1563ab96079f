# round 4 call E: the register-resident chaining filter walk (tests, C3 partitioned + ordered bench
# lines), and the split with its stores written linearly (tuning build, timing only)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4e_ab.log && \
timeout -k 10 400 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3" > gpurun_out/r4e_tests.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4e_c3.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4e_c3ord.log 2>&1 && \
for v in "CCJ_ABLATE=16384" "CCJ_ABLATE=0"; do \
  env $v timeout -k 10 100 python -u bench.py --lib tuning --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4e_run.log 2>&1 || exit 1; \
  echo "$v $(tail -1 gpurun_out/r4e_run.log)" >> gpurun_out/r4e_ab.log; \
done
