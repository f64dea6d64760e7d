# Llama-2-7B preset breakdown + per-kernel hipBLASLt stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
python tools/gpu_job.py prof --set preset=llama2_7b_fsdp_mp --set kgrep=Cijk --tag l2p > /dev/null 2>&1 || exit 5
cat gpurun_out/l2p/kstats.log; head -24 gpurun_out/l2p/breakdown.log
