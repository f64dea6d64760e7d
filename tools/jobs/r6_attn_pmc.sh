# Attention kernels after the XCD-aware order: L2 hit rate and MFMA busy at the headline shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6attnpmc
P1="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P3="SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P3"; do
  i=$((i+1))
  for sh in llama3-8B-B40; do
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/r6attnpmc/p${i}_$sh -o p -- python3 tools/bench_attn.py --shapes $sh --iters 3 > gpurun_out/r6attnpmc/p${i}_$sh.log 2>&1 || { echo "pmc pass $i $sh failed"; tail -5 gpurun_out/r6attnpmc/p${i}_$sh.log; exit 4; }
  done
done
python tools/pmc_db_summary.py $(find gpurun_out/r6attnpmc -name "*.db") --filter attn > gpurun_out/r6attnpmc/summary.txt 2>&1
cat gpurun_out/r6attnpmc/summary.txt
find gpurun_out/r6attnpmc -name "*.db" -delete
