#!/bin/bash
# round-3 final, part 3: PMC passes on the bench (FETCH_SIZE; MFMA busy cycles), each its own run
set -o pipefail
bash tools/gpu_pmc.sh r03f3_fetch || exit $?
bash tools/gpu_pmc_sq.sh r03f3_sq SQ_VALU_MFMA_BUSY_CYCLES,GRBM_GUI_ACTIVE,SQ_INSTS_VALU_MFMA_MOPS_F16,SQ_INSTS_VALU_MFMA_MOPS_I8 || exit $?
