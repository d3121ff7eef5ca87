# Round profile on the box: probes, rocprof kernel stats + PMC traffic, default bench line.
# usage: bash tools/gpu_profile.sh <tag>; then locally: python tools/pmc_traffic.py <tag> 24
set -o pipefail
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 60 ./tools/mb_mfma > gpurun_out/${TAG}_mb_mfma.txt 2>&1 || exit 1
bash tools/profile_bench.sh ${TAG} || { tail -20 gpurun_out/prof_${TAG}.err; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
echo done
