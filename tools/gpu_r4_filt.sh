# round 4: the chaining filter walk (tests + C3 bench), then split ablations on the C2 bench (tuning build)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py -x -v --timeout 300 --timeout-method thread -k "chain" > gpurun_out/r4f_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4f_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4f_c2.log 2>&1 && \
for ab in 0 16 32 48 8224 8240; do \
  CCJ_ABLATE=$ab timeout -k 10 200 python -u bench.py --lib tuning --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4f_abl_$ab.log 2>&1 || exit 1; \
done
