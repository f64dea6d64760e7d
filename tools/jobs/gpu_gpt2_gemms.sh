# Per-kernel hipBLASLt stats of the GPT-2 preset (which GEMM solutions run, how long each takes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
python tools/gpu_job.py prof --set preset=gpt2_774m_ddp --set kgrep=Cijk --tag g2gemm > /dev/null 2>&1 || exit 5
cat gpurun_out/g2gemm/kstats.log
