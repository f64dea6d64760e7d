# all BASELINE configs on one box, back to back (same-box snapshot)
set -o pipefail
mkdir -p gpurun_out/presets
for cfg in llama3_8b_fsdp:"" gpt2_774m_ddp:"--preset gpt2_774m_ddp" llama32_1b_lora_alpaca:"--preset llama32_1b_lora_alpaca" llama2_7b_fsdp_mp:"--preset llama2_7b_fsdp_mp"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 500 python -u bench.py $args --steps 10 --warmup 3 > gpurun_out/presets/$name.log 2>&1 || { tail -20 gpurun_out/presets/$name.log; exit 1; }
  tail -1 gpurun_out/presets/$name.log | cut -c1-200
done
