#!/bin/bash
# B=4 shard: kNN split policy variants (default: split C=128 only; never split; split every C), 3 rounds interleaved
set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
for r in 1 2 3; do
for lib in dgcnn.pytorch_amd/dgx/libdgx.so tools/diag/libdgx_nosplit.so tools/diag/libdgx_allsplit.so tools/diag/libdgx_base.so; do
  echo -n "round $r $(basename $lib) B=4: "
  DGX_LIB=$(realpath $lib) timeout -k 10 200 python3 bench.py --batch 4 --no-cpu-baseline --no-eager-baseline --no-posemb-leg --no-edgeconv-leg --no-attention-leg --no-fp32-leg --steps 50 --warmup 10 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d.get("roofline",{}).get("knn_ms_by_layer"))' || exit 1
done
done
