# Round-2: HIP-graph decode step: tests + decode benchmark (graph on / off).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread -k "decode or graph" > gpurun_out/graph_tests.log 2>&1 && \
for M in "llama3 8B" "GPT2 774M" "GPT2 124M" "llama3_2 1B"; do
  set -- $M
  timeout -k 10 200 python tools/bench_decode.py --model $1 --num_params $2 --graph 1 >> gpurun_out/r2_decode_graph.log 2>&1 || exit 1
  timeout -k 10 200 python tools/bench_decode.py --model $1 --num_params $2 --graph 0 >> gpurun_out/r2_decode_graph.log 2>&1 || exit 1
done
