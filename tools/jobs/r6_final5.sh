# final round-6 tree after the hd-64 tiling rule: GPU suite, smoke, LoRA preset (hd 64, no dropout)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6final5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6final5/tests.log 2>&1 || { tail -40 gpurun_out/r6final5/tests.log; exit 5; }
tail -1 gpurun_out/r6final5/tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6final5/smoke.log 2>&1 || { tail -20 gpurun_out/r6final5/smoke.log; exit 6; }
tail -2 gpurun_out/r6final5/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --preset llama32_1b_lora_alpaca > gpurun_out/r6final5/bench_lora.log 2>&1 || { tail -20 gpurun_out/r6final5/bench_lora.log; exit 7; }
tail -1 gpurun_out/r6final5/bench_lora.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*\|"mfu": [0-9.]*' | tr '\n' ' '; echo
