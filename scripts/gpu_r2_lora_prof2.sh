# LoRA Alpaca preset: rocprof DB kept for per-dispatch analysis
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/lora2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/lora2 -o run -- python3 $R/bench.py --preset llama32_1b_lora_alpaca --steps 2 --warmup 2 > $R/gpurun_out/lora2/log.txt 2>&1
