# PMC passes over the attention kernels at the Llama-3-8B / GPT-2 shapes (tools/bench_attn.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_attn
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d /tmp/pa1 -o p1 -- python3 $R/tools/bench_attn.py --iters 3 > $R/gpurun_out/pmc_attn/p1.log 2>&1 && \
python3 $R/tools/pmc_summary.py $(ls /tmp/pa1/*counter_collection.csv) --filter attn > $R/gpurun_out/pmc_attn/p1_summary.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --output-format csv -d /tmp/pa2 -o p2 -- python3 $R/tools/bench_attn.py --iters 3 > $R/gpurun_out/pmc_attn/p2.log 2>&1 && \
python3 $R/tools/pmc_summary.py $(ls /tmp/pa2/*counter_collection.csv) --filter attn > $R/gpurun_out/pmc_attn/p2_summary.txt 2>&1
