set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_lora.py --tokens 9216 --iters 50 > gpurun_out/bench_lora_9k.jsonl 2>&1 || { tail -20 gpurun_out/bench_lora_9k.jsonl; exit 1; }
cat gpurun_out/bench_lora_9k.jsonl
