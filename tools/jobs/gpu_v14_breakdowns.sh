# v14 kernel-trace breakdowns of the final round-5 tree: headline Llama-3-8B and GPT2-774M
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/v14
timeout -k 10 900 python tools/gpu_job.py prof --tag v14/headline > gpurun_out/v14/headline.log 2>&1 || { tail -30 gpurun_out/v14/headline.log; exit 5; }
head -22 gpurun_out/v14/headline/breakdown.log
timeout -k 10 900 python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --tag v14/gpt2 > gpurun_out/v14/gpt2.log 2>&1 || { tail -30 gpurun_out/v14/gpt2.log; exit 6; }
head -22 gpurun_out/v14/gpt2/breakdown.log
