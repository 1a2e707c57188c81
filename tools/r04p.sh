#!/bin/bash
# Scatter timing decomposition: kernel traces of the cfg2 step and the B=4 shard
# with the shipped library and the probe builds (sp1: no edge loop, sp4: no
# degree sort; results of sp1 are not gradients, timing only).
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
for lib in dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_sp1.so tools/diag/libdgx_sp4.so; do
  for b in 32 4; do
    tag=r04p_$(basename $lib .so)_b$b
    DGX_LIB=$(realpath $lib) KT_ONLY=1 timeout -k 10 200 bash tools/profile.sh $tag --batch $b --steps 5 --warmup 2 > gpurun_out/$tag.log 2>&1 || { tail gpurun_out/$tag.log; exit 1; }
    echo "== $tag"; grep -E "scatter|rev_graph" gpurun_out/prof_$tag/kt_summary.txt
  done
done
