# Per-kernel stats of the LoRA preset: hipBLASLt solutions and PyTorch elementwise kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
python tools/gpu_job.py prof --set preset=llama32_1b_lora_alpaca --set kgrep=Cijk --tag lgemm > /dev/null 2>&1 || exit 5
head -40 gpurun_out/lgemm/kstats.log
