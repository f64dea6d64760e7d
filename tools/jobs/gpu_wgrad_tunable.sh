# dW GEMM: our MFMA kernel vs the best hipBLASLt / rocBLAS solution TunableOp finds for the
# token-major layout (every candidate timed), Llama-3-8B shapes at 40,960 tokens
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/wgtune
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/wgtune/tuned%d.csv \
  timeout -k 10 900 python -u tools/bench_wgrad.py --tokens 40960 --models llama3_8b --rounds 3 > gpurun_out/wgtune/llama.jsonl 2>&1 || { tail -5 gpurun_out/wgtune/llama.jsonl; exit 3; }
grep -o '"gemm": "[a-z_]*"\|"hipblaslt_tflops": [0-9.]*\|"mfma_tflops": [0-9.]*' gpurun_out/wgtune/llama.jsonl | paste - - -
