set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --actv_ckpt none --batch_size 24 --steps 10 --warmup 3 > gpurun_out/extra_none_b24.log 2>&1 || { tail -20 gpurun_out/extra_none_b24.log; exit 1; }
tail -1 gpurun_out/extra_none_b24.log | cut -c1-250
timeout -k 10 500 python -u bench.py --actv_ckpt selective --batch_size 24 --steps 10 --warmup 3 > gpurun_out/extra_sel_b24.log 2>&1 || { tail -20 gpurun_out/extra_sel_b24.log; exit 1; }
tail -1 gpurun_out/extra_sel_b24.log | cut -c1-250
timeout -k 10 500 python -u bench.py --preset llama32_1b_lora_alpaca --steps 10 --warmup 3 > gpurun_out/extra_lora.log 2>&1 || { tail -20 gpurun_out/extra_lora.log; exit 1; }
tail -1 gpurun_out/extra_lora.log | cut -c1-250
