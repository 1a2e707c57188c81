#!/bin/bash
# Final-tree refresh (round 6): PMC passes of the default cfg2 step, the cfg3 /
# cfg5 / 4-cloud bench lines and a 4-cloud kernel trace; logs under gpurun_out/.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT" || exit 1
NOL="--no-roofline-leg --no-fp32-leg --no-edgeconv-leg --no-posemb-leg --no-attention-leg --no-cpu-baseline"
bash tools/profile.sh r09x > gpurun_out/r09x_profile.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/r09x_profile.log; exit 1; }
tail -3 gpurun_out/r09x_profile.log
bash tools/gpu_run.sh 300 \
  "r09x_bench_cfg3.log::python -u bench.py --config cfg3 --steps 10 --warmup 3 $NOL --no-eager-baseline" \
  "r09x_bench_cfg5.log::python -u bench.py --config cfg5 --steps 10 --warmup 3 $NOL --no-eager-baseline" \
  "r09x_bench_b4.log::python -u bench.py --batch 4 --steps 50 --warmup 10 $NOL" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/r09x_b4_prof" -o run -- python3 "$ROOT/bench.py" --batch 4 --steps 20 \
    --warmup 5 $NOL --no-eager-baseline > "$ROOT/gpurun_out/r09x_b4_prof.log" 2>&1 || { echo "b4 trace failed"; exit 1; }
KS=$(find "$ROOT/gpurun_out/r09x_b4_prof" -name run_kernel_stats.csv -print -quit)
python3 "$ROOT/tools/kt_summary.py" "$(dirname "$KS")" 13 > "$ROOT/gpurun_out/r09x_b4_kernel_stats.txt" && head -8 "$ROOT/gpurun_out/r09x_b4_kernel_stats.txt"
echo done
