#!/bin/bash
# attention kernels: causal vs non-causal vs long T timings, then PMC passes on the Llama-3-8B B=24 shape
set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_attn.py --iters 30 --shapes llama3-8B-B24,gpt2-774M-nodrop > gpurun_out/pmc2/t_causal.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_attn.py --iters 30 --shapes llama3-8B-B24,gpt2-774M-nodrop --noncausal > gpurun_out/pmc2/t_noncausal.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_attn.py --iters 20 --shapes llama3-8B-B24 --T 4096 > gpurun_out/pmc2/t_4k.log 2>&1 || exit 1
grep shape gpurun_out/pmc2/t_*.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d /tmp/pmc$i -o run -- python3 tools/bench_attn.py --iters 10 --shapes llama3-8B-B24 > gpurun_out/pmc2/p$i.log 2>&1 || { tail -5 gpurun_out/pmc2/p$i.log; exit 1; }
  python tools/pmc_summary.py $(find /tmp/pmc$i -name "*counter_collection.csv") --filter attn > gpurun_out/pmc2/p${i}_summary.txt || exit 1
done
cat gpurun_out/pmc2/p*_summary.txt
