# round 5 call T: the split's keys by 16-byte loads (K16 form) — probe / C3 / multi-GPU tests, then
# C2 and C3 A/B against the 8-byte build (interleaved)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_probe_gpu.py tests/test_c3_gpu.py tests/test_dist_gpu.py > gpurun_out/r5t_tests.log 2>&1 && \
bash tools/gpu_ab.sh r5k16s c2 3 product tools/abx/libccj_k8.so > gpurun_out/r5k16s_ab.log 2>&1 && \
bash tools/gpu_ab.sh r5k16c c3split 2 product tools/abx/libccj_k8.so > gpurun_out/r5k16c_ab.log 2>&1
