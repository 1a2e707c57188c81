#!/bin/bash
# Round profiling bundle on the GPU box: kernel trace + PMC passes of bench.py
# for each config (tools/profile.sh), then the B=4 strong-scaling shard line.
# usage: tools/round_profiles.sh <round-tag> <config>...
set -o pipefail
TAG=$1; shift
for cfg in "$@"; do
    echo "== $cfg"
    timeout -k 10 900 bash tools/profile.sh "${TAG}_$cfg" --config "$cfg" --steps 10 --warmup 3 \
        > "gpurun_out/${TAG}_${cfg}_profile.log" 2>&1 || { echo "profile $cfg failed"; tail -20 "gpurun_out/${TAG}_${cfg}_profile.log"; exit 1; }
    tail -3 "gpurun_out/${TAG}_${cfg}_profile.log"
done
echo "profiles done"
