# PMC passes (one per counter group) over the dW kernel on the Llama-3-8B shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc/p1 -o p1 -- python3 $R/tools/bench_wgrad.py --models llama3_8b --variants 1 --rounds 1 --iters 3 > $R/gpurun_out/pmc/p1.log 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc/p2 -o p2 -- python3 $R/tools/bench_wgrad.py --models llama3_8b --variants 1 --rounds 1 --iters 3 > $R/gpurun_out/pmc/p2.log 2>&1
