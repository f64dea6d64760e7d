# SwiGLU loads-in-flight A/B, then the full GPU suite + smoke() + the GPT-2 and Llama-2 presets
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/val1
timeout -k 10 240 python -u tools/bench_swiglu_u.py > gpurun_out/val1/swiglu_u.jsonl 2>&1 || { tail -20 gpurun_out/val1/swiglu_u.jsonl; exit 2; }
cat gpurun_out/val1/swiglu_u.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/val1/pytest.log 2>&1 || { tail -40 gpurun_out/val1/pytest.log; exit 3; }
tail -2 gpurun_out/val1/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val1/smoke.log 2>&1 || { tail -20 gpurun_out/val1/smoke.log; exit 4; }
grep "smoke ok" gpurun_out/val1/smoke.log
for p in gpt2_774m_ddp llama2_7b_fsdp_mp; do
  timeout -k 10 400 python -u bench.py --preset $p --steps 20 --warmup 5 > gpurun_out/val1/$p.log 2>&1 || { tail -20 gpurun_out/val1/$p.log; exit 5; }
  echo "$p $(tail -1 gpurun_out/val1/$p.log | grep -o '"value": [0-9.]*\|"sclk_mhz_avg": [0-9.]*' | tr '\n' ' ')"
done
