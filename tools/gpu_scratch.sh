set -o pipefail
mkdir -p gpurun_out
ZK_T33_OCT64_MIN=4 bash tools/gpu_trace.sh | grep "zk step [0-4]"
REPS="1 2 3 4" bash tools/gpu_ab_env.sh ZK_T33_OCT64_MIN=1 ZK_T33_OCT64_MIN=4
