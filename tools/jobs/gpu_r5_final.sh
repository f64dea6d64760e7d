# Final tree on one box: full GPU suite, smoke(), headline bench (driver settings), LoRA / GPT-2 presets
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest.log 2>&1 || { tail -40 gpurun_out/final/pytest.log; exit 3; }
tail -1 gpurun_out/final/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 4; }
grep -c "smoke ok" gpurun_out/final/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final/headline.log 2>&1 || { tail -20 gpurun_out/final/headline.log; exit 5; }
echo "headline $(tail -1 gpurun_out/final/headline.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
for p in llama32_1b_lora_alpaca gpt2_774m_ddp; do
  timeout -k 10 400 python -u bench.py --preset $p --steps 20 --warmup 5 > gpurun_out/final/$p.log 2>&1 || { tail -20 gpurun_out/final/$p.log; exit 6; }
  echo "$p $(tail -1 gpurun_out/final/$p.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
done
