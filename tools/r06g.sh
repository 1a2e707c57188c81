#!/bin/bash
# round 5, session g: kNN lab — FIFO capacity / flush trigger variants, fix-up mask
set -o pipefail
mkdir -p gpurun_out
for v in q24 q20 q16; do
  timeout -k 10 120 ./tools/knn_lab_$v 20 > gpurun_out/r06g_lab_$v.log 2>&1; rc=$?; echo "== $v"; cat gpurun_out/r06g_lab_$v.log; [ $rc -eq 0 ] || exit 1
done
