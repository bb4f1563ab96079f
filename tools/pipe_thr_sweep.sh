#!/bin/bash
# Threshold sweep + dynamic tuner on main.cpp's default pipeline shape (run on the GPU box).
set -o pipefail
BIN=chunk-compaction-in-vectorized-execution-simd_amd/host/ccj_pipeline
ARGS="--join-num 3 --chunk-factor 1 --lhs-size 20000000 --rhs-size 2000000 --engine batched"
for t in chain lp; do for b in 256 2048; do
  for thr in "1,1,1" "32,32,32" "64,64,64" "128,128,128" "$((b/2)),$((b/2)),$((b/2))" "$b,$b,$b"; do
    echo "== $t B=$b thresholds=$thr"
    timeout -k 10 120 $BIN $ARGS --table $t --block-size $b --compact full --thresholds $thr --repeat 8 2>&1 | grep -E "TIMES|PIPE|\[join" || exit 1
  done
  echo "== $t B=$b dynamic"
  timeout -k 10 300 $BIN $ARGS --table $t --block-size $b --compact dynamic --repeat 150 2>&1 | grep -E "PIPE|TUNER|\[join" || exit 1
done; done
