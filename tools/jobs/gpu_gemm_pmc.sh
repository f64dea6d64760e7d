# PMC of our dW kernel vs our forward-layout kernel vs hipBLASLt on the Llama-3-8B o-projection
# shape (4096 x 4096, 40,960 tokens): where the dW kernel's cycles go
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/gemmpmc
P1="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/gemmpmc/w$i -o w$i -- python3 tools/bench_wgrad.py --tokens 40960 --models llama3_8b --only o --rounds 1 --iters 3 --no_hipblaslt > gpurun_out/gemmpmc/w$i.log 2>&1 || { echo "wgrad pmc $i failed"; tail -5 gpurun_out/gemmpmc/w$i.log; exit 3; }
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/gemmpmc/n$i -o n$i -- python3 tools/bench_gemm_nt.py --models llama --only o --rounds 1 --iters 3 > gpurun_out/gemmpmc/n$i.log 2>&1 || { echo "nt pmc $i failed"; tail -5 gpurun_out/gemmpmc/n$i.log; exit 4; }
done
python tools/pmc_db_summary.py $(find gpurun_out/gemmpmc -name "*.db") --filter "" > gpurun_out/gemmpmc/summary.txt 2>&1
grep -A40 "wgrad4\|gemm_nt4p\|Cijk" gpurun_out/gemmpmc/summary.txt | head -150
find gpurun_out/gemmpmc -name "*.db" -delete
