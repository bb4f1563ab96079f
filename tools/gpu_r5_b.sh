# round 5 call B: the tests of this round's changes; the split's stores with its key reads beside
# them (is the split bound by HBM time: scattered writes + linear reads?); the C3 filter walk with
# its per-partition workgroup rotation against the fixed assignment; scalar-path reads last
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_probe_gpu.py::test_ordered_probe_small_inputs_equal_chunk_probe" \
  "tests/test_probe_gpu.py::test_partitioned_probe_skew_few_tiles_stays_one_pass" \
  tests/test_known_answers_gpu.py::test_reference_sum_vector_on_gpu tests/test_dist_gpu.py \
  "tests/test_probe_gpu.py::test_partitioned_chaining_c3_skew" tests/test_c3_gpu.py \
  "tests/test_bench_gpu.py::test_bench_c2_with_other_paths" > gpurun_out/r5b_tests.log 2>&1 && \
( for a in "22 1 both 512 8" "22 1 read 512 8" "44 1 both 256 8" "44 1 read 256 8" "64 1 read 176 8" "11 1 read 1024 8"; do
    timeout -k 5 60 ./tools/runstore $a || exit 1; done ) > gpurun_out/r5b_runstore.log 2>&1 && \
bash tools/gpu_ab.sh r5rot c3split 2 product tools/abx/libccj_norot.so > gpurun_out/r5rot_ab.log 2>&1 && \
bash tools/gpu_ab.sh r5rotc3 c3 2 product tools/abx/libccj_norot.so > gpurun_out/r5rotc3_ab.log 2>&1 && \
( for m in "sca 8" "vec 0" "mix 4" "mix 8" "mix 16"; do timeout -k 5 60 ./tools/sreq $m || exit 1; done ) > gpurun_out/r5b_sreq.log 2>&1
