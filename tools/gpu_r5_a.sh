# round 5 first GPU call: the store-pattern microbenchmark, then the tests of this round's changes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_r5_runstore.sh && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_probe_gpu.py::test_ordered_probe_small_inputs_equal_chunk_probe" \
  "tests/test_probe_gpu.py::test_partitioned_probe_skew_few_tiles_stays_one_pass" \
  tests/test_known_answers_gpu.py::test_reference_sum_vector_on_gpu tests/test_dist_gpu.py \
  "tests/test_bench_gpu.py::test_bench_c2_with_other_paths" > gpurun_out/r5a_tests.log 2>&1
cd $GRAFT_REPO_ROOT && bash tools/gpu_ab.sh r5def c2 2 tuning tools/abx/libccj_defer.so tuning:CCJ_SPLIT_PER=10 tools/abx/libccj_defer.so:CCJ_SPLIT_PER=10 > gpurun_out/r5def_ab.log 2>&1
