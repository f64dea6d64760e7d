#!/bin/bash
# PMC passes on the dW GEMM kernel (Llama-3-8B shapes, variant 2)
set -o pipefail
mkdir -p gpurun_out/pmc_wg
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_SALU"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/pw$i -o run -- python3 tools/bench_wgrad.py --models llama3_8b --variants 2 --rounds 1 --iters 3 > gpurun_out/pmc_wg/p$i.log 2>&1 || { tail -5 gpurun_out/pmc_wg/p$i.log; exit 1; }
  python tools/pmc_summary.py $(find /tmp/pw$i -name "*counter_collection.csv") --filter wgrad > gpurun_out/pmc_wg/p${i}_summary.txt || exit 1
done
cat gpurun_out/pmc_wg/p*_summary.txt
