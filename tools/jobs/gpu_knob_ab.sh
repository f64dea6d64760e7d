# Same-box A/B of the shipped A/B switches on the GPT-2 and LoRA presets (two runs each, interleaved).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/knob
run() {  # tag preset env...
  local tag=$1 preset=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --preset $preset --steps 10 --warmup 3 > gpurun_out/knob/${tag}.log 2>&1 || exit 3
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/knob/${tag}.log)"
}
for i in 1 2; do
run gpt2_base_$i gpt2_774m_ddp BLLM_X=1
run gpt2_wgradlt_$i gpt2_774m_ddp BLLM_WGRAD_GEMM=0
run gpt2_nodwt_$i gpt2_774m_ddp BLLM_DGRAD_WT=0
run lora_base_$i llama32_1b_lora_alpaca BLLM_X=1
run lora_nodwt_$i llama32_1b_lora_alpaca BLLM_DGRAD_WT=0
done
