# Round 4: per-step timeline and per-block phases of the MFMA steps (epilogue costs).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_trace.sh || exit 1
STEPS="1 2 3 4" bash tools/gpu_blocks.sh || exit 1
exit 0
