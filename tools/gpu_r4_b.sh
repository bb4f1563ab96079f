# round 4 call B: split ablations and two-workgroups-per-CU split variants on the C2 bench (tuning
# build; phases.hash_find_bucket_ms is the split), then the product line for comparison
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4b_*.log && \
for v in "CCJ_ABLATE=0" "CCJ_ABLATE=16" "CCJ_ABLATE=32" "CCJ_ABLATE=48" "CCJ_ABLATE=8224" "CCJ_ABLATE=8240" "CCJ_SPLIT_T=512" "CCJ_SPLIT_T=1025" "CCJ_SPLIT_T=512 CCJ_ABLATE=48"; do \
  env $v timeout -k 10 200 python -u bench.py --lib tuning --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4b_run.log 2>&1 || exit 1; \
  echo "$v $(tail -1 gpurun_out/r4b_run.log)" >> gpurun_out/r4b_ab.log; \
done && \
timeout -k 10 200 python -u bench.py --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4b_product.log 2>&1
