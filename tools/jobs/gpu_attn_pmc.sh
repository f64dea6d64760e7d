# Attention kernels: timing at the headline / GPT-2 shapes, then two PMC passes (SQ counters)
# over one fwd + bwd of the headline shape, to see where the cycles of each kernel go.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/attnpmc
timeout -k 10 200 python -u tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64,gpt2-774M-B64-nodrop > gpurun_out/attnpmc/time.jsonl 2>&1 || { tail -5 gpurun_out/attnpmc/time.jsonl; exit 3; }
cat gpurun_out/attnpmc/time.jsonl
P1="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/attnpmc/p$i -o p$i -- python3 tools/bench_attn.py --shapes llama3-8B-B40,gpt2-774M-B64 --iters 3 > gpurun_out/attnpmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/attnpmc/p$i.log; exit 4; }
done
python tools/pmc_summary.py $(find gpurun_out/attnpmc -name "*counter_collection.csv") --filter attn > gpurun_out/attnpmc/summary.txt 2>&1
cat gpurun_out/attnpmc/summary.txt
