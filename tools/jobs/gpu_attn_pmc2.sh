# Attention kernels (fwd, dK/dV, dQ): per-kernel SQ counters at the headline and GPT-2 shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/attnpmc2
P1="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P3="SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  for sh in llama3-8B-B40 gpt2-774M-B64; do
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/attnpmc2/p${i}_$sh -o p -- python3 tools/bench_attn.py --shapes $sh --iters 3 > gpurun_out/attnpmc2/p${i}_$sh.log 2>&1 || { echo "pmc pass $i $sh failed"; tail -5 gpurun_out/attnpmc2/p${i}_$sh.log; exit 4; }
  done
done
for sh in llama3-8B-B40 gpt2-774M-B64; do
  echo "== $sh"
  python tools/pmc_db_summary.py $(find gpurun_out/attnpmc2 -path "*_$sh/*" -name "*.db") --filter attn
done > gpurun_out/attnpmc2/summary.txt 2>&1
cat gpurun_out/attnpmc2/summary.txt
find gpurun_out/attnpmc2 -name "*.db" -delete
