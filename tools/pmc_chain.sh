#!/bin/bash
# PMC passes over the training chain alone (shape_probe, 128 trees, prepared batch
# reused): wave-state counters, HBM traffic and L2 hit rate per kernel, one pass each.
#   bash tools/pmc_chain.sh gpurun_out/pmc_chain
set -eo pipefail
OUT=${1:-gpurun_out/pmc_chain}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
P="python tools/shape_probe.py --only mean --steps 20"
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/p$i" -- $P > "$OUT/p$i.log" 2>&1
done
echo done
