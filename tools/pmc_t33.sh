#!/bin/bash
# Round 6: the same SQ counters on the first k_gkr_t33 (the
# bench's proofs, steps launched one at a time) and on its memory-only W8
# pattern (tools/mb_order: k_order<STRIDE, 2 ahead, stores>, the kernel's own
# addressing and prefetch depth), in two passes of <= 8 SQ counters each.
# Summary: python3 tools/pmc_t33_summary.py gpurun_out/pmct33_*
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fold --no-e2e --no-serving --no-circuit --no-config5 --no-config4 --no-plain"
export ZK_PRELAUNCH=0
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_WAIT_ANY"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmct33_k$i -o run -- $B > /dev/null 2> gpurun_out/pmct33_k$i.err || { tail -5 gpurun_out/pmct33_k$i.err; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmct33_m$i -o run -- ./tools/mb_order > /dev/null 2> gpurun_out/pmct33_m$i.err || { tail -5 gpurun_out/pmct33_m$i.err; exit 1; }
done
echo pmc ok
