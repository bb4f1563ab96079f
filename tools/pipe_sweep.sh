#!/bin/bash
# sweep the batched pipeline: table kind x compaction x block size at main.cpp's default shape
set -o pipefail
BIN=chunk-compaction-in-vectorized-execution-simd_amd/host/ccj_pipeline
for t in chain lp; do for b in 256 2048; do for c in none full; do
  echo "== $t B=$b compact=$c"
  timeout -k 10 300 $BIN --join-num 3 --chunk-factor 1 --lhs-size 20000000 --rhs-size 2000000 --table $t --compact $c --block-size $b --engine batched --repeat 3 2>&1 | grep -v ROW || exit 1
done; done; done
for c in 0 2; do echo "== ref chain compact=$c"; timeout -k 10 300 oracle/_ref/ref_driver pipeline chain 256 3 1 20000000 2000000 $c 1 || exit 1; done
echo "== ref probe"; timeout -k 10 300 oracle/_ref/ref_driver bench lp next 2048 67108864 1 134217728 67108864 42
