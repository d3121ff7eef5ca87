#!/bin/bash
# SQ counters of the proof's steps (separate passes, <= 8 SQ counters each; steps launched one at a time)
# usage: bash tools/pmc_steps.sh; then python tools/pmc_summary.py --steps gpurun_out/pmc_s1 gpurun_out/pmc_s2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-config4"
export ZK_PRELAUNCH=0
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_s1 -o run -- $B > /dev/null 2> gpurun_out/pmc_s1.err || { tail -5 gpurun_out/pmc_s1.err; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_s2 -o run -- $B > /dev/null 2> gpurun_out/pmc_s2.err || { tail -5 gpurun_out/pmc_s2.err; exit 1; }
echo pmc ok
