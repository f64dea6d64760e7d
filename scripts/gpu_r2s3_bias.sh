set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bias_tests.log 2>&1 || { tail -30 gpurun_out/bias_tests.log; exit 1; }
tail -2 gpurun_out/bias_tests.log
timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/bench_bias_gpt2.log 2>&1 || exit 1
tail -1 gpurun_out/bench_bias_gpt2.log | cut -c1-300
BLLM_FUSED_BIAS=0 timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/bench_bias_gpt2_off.log 2>&1 || exit 1
tail -1 gpurun_out/bench_bias_gpt2_off.log | cut -c1-300
timeout -k 10 600 python -u bench.py --preset gpt2_774m_ddp --steps 10 --warmup 3 > gpurun_out/bench_bias_gpt2_b.log 2>&1 || exit 1
tail -1 gpurun_out/bench_bias_gpt2_b.log | cut -c1-300
mkdir -p gpurun_out/ovl
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/ovl/db_fsdp -o run -- python3 $R/bench.py --force_comm --steps 2 --warmup 2 > $R/gpurun_out/ovl/fsdp.log 2>&1 || { tail -20 $R/gpurun_out/ovl/fsdp.log; exit 1; }
python3 $R/tools/overlap.py $R/gpurun_out/ovl/db_fsdp/run_results.db --md $R/gpurun_out/ovl/fsdp_overlap.md
cd $R
for b in 40 56 64; do
  timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --batch_size $b > gpurun_out/bsweep_b$b.log 2>&1 || exit 1
  tail -1 gpurun_out/bsweep_b$b.log | cut -c1-260
done
