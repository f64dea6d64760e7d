set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_nt or bias_grad or gelu or dropout" > gpurun_out/kt.log 2>&1 || echo "tests rc=$?" >> gpurun_out/kt.log
grep -q "passed" gpurun_out/kt.log && ! grep -qi "fault\|core dumped\|Aborted" gpurun_out/kt.log || exit 5
timeout -k 10 400 python -u tools/bench_gemm_nt.py --arms hipblaslt,gemm_nt --rounds 3 --iters 10 > gpurun_out/sv_ab.jsonl 2> gpurun_out/sv_ab.err || exit 6
timeout -k 10 120 python -u tools/bench_ew.py > gpurun_out/ew.json 2>&1 || exit 7
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_down1 -o pmc --output-format csv -- python tools/bench_gemm_nt.py --only down --arms hipblaslt,gemm_nt --rounds 1 --iters 4 > gpurun_out/pmc1.log 2>&1 || exit 8
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA FETCH_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_down2 -o pmc --output-format csv -- python tools/bench_gemm_nt.py --only down --arms hipblaslt,gemm_nt --rounds 1 --iters 4 > gpurun_out/pmc2.log 2>&1 || exit 9
