#!/bin/bash
# every bench preset once (1 GPU), summary lines to stdout
set -o pipefail
mkdir -p gpurun_out
for p in llama3_8b_fsdp gpt2_774m_ddp llama32_1b_lora_alpaca llama2_7b_fsdp_mp; do
  timeout -k 10 500 python -u bench.py --preset $p --steps 10 --warmup 3 > gpurun_out/preset_$p.log 2>&1 || { tail -20 gpurun_out/preset_$p.log; exit 1; }
  tail -1 gpurun_out/preset_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['metric'], d['value'], d['ms_per_step'], d.get('mfu'), d.get('peak_mem_gib'))"
done
