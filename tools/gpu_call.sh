# round 5 call AO: C5 with the payload rows in fine-grained (1) / uncached (3) memory (tuning build,
# CCJ_PAY_ALLOC): gather time A/B, then the gather's L2->fabric read requests by size per allocation
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5ao c5 2 tuning tuning:CCJ_PAY_ALLOC=1 tuning:CCJ_PAY_ALLOC=3 > gpurun_out/r5ao_ab.log 2>&1 && \
for a in 0 3; do
  CCJ_PAY_ALLOC=$a timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum \
    --kernel-include-regex gather_payload -d gpurun_out/r5ao_pmc_$a -o pmc --output-format csv -- \
    python3 bench.py --lib tuning --workload c5 --no-cpu --no-other --no-other-workloads --no-verify --steps 2 --warmup 1 \
    > gpurun_out/r5ao_pmc_$a.log 2>&1 || exit 1
done
